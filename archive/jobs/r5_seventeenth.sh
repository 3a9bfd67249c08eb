# Round 5, seventeenth box: RandomResizedCrop with the column-major LDS resampling (a wave per 64 output
# columns of a row, horizontal taps held per band) against the row-major form (impl="lds_rows"): bit-exact
# tests, kernel timings, LDS counters, and the resident loader with on-device augmentation.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 rrc_tests python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k random_resized_crop
run 300 kbench python benchmarks/kernels_bench.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 400 pmc_insts rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc3 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 60 pmc_summary python tools/pmc_summary.py gpurun_out/pmc_summary_rrc.json gpurun_out/pmc3
run 300 res_u8_aug python benchmarks/bench_resident.py --dtype uint8 --augment
