# RandomResizedCrop fast LDS path: exactness tests, timing, PMC pass.
source tools/gpu_job.sh
run 300 rrc_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "random_resized or augment"
run 300 kbench python benchmarks/kernels_bench.py
rm -rf gpurun_out/pmc_rrc_a
run 90 pmc_rrc_a timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/pmc_rrc_a -o k --output-format csv -- python3 tools/rrc_probe.py
