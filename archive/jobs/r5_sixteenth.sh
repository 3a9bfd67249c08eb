# Round 5, sixteenth box: the kernel benchmark on the final tree, and its hardware counters, one rocprofv3
# --pmc pass per counter group (kernel trace only, no other trace domain): HBM bytes, waves / busy cycles,
# instruction mix and LDS bank conflicts; then the per-kernel summary. Also the train + eval example on the GPU.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 kbench python benchmarks/kernels_bench.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 400 pmc_fetch rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc1 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 400 pmc_write rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc2 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 400 pmc_insts rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc3 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 60 pmc_summary python tools/pmc_summary.py gpurun_out/pmc_summary.json gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
run 200 example_gpu python examples/torch_dataset.py --epochs 3
