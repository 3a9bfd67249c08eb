source tools/gpu_job.sh
run 300 kbench python benchmarks/kernels_bench.py
rm -rf gpurun_out/pmc_a gpurun_out/pmc_b gpurun_out/pmc_c
run 300 pmc_a timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_a -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 300 pmc_b timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_b -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 300 pmc_c timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace -d gpurun_out/pmc_c -o k --output-format csv -- python3 benchmarks/kernels_bench.py
