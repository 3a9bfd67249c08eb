source tools/gpu_job.sh
run 400 ktests python -u -m pytest tests/test_kernels_gpu.py tests/test_loader_gpu.py tests/test_tokens.py -x -q --timeout 120 --timeout-method thread -m gpu
run 300 kbench python benchmarks/kernels_bench.py
run 120 pw_window python benchmarks/bench_pointwise.py --dispatch window
run 120 pw_window_groups python benchmarks/bench_pointwise.py --dispatch window --consumer groups
run 120 pw_inline python benchmarks/bench_pointwise.py --dispatch inline
run 180 tokk_8_pad python benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 4 --mode pad --batches-per-window 8
run 180 tokk_8_idle python benchmarks/bench_tokens.py --steps 1000 --warmup 100 --idle-steps 300 --producers 4 --batches-per-window 8
rm -rf gpurun_out/pmc_split
run 200 pmc_split timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/pmc_split -o k --output-format csv -- python3 benchmarks/kernels_bench.py
