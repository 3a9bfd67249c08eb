source tools/gpu_job.sh
run 300 kbench python benchmarks/kernels_bench.py
run 400 pmc_fetch rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc1 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 400 pmc_write rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc2 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
