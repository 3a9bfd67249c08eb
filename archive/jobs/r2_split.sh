source tools/gpu_job.sh
run 400 ktests python -u -m pytest tests/test_kernels_gpu.py tests/test_loader_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu
run 300 kbench python benchmarks/kernels_bench.py
run 120 pw_window python benchmarks/bench_pointwise.py --dispatch window
run 120 pw_window_groups python benchmarks/bench_pointwise.py --dispatch window --consumer groups
run 120 pw_inline python benchmarks/bench_pointwise.py --dispatch inline
run 200 tpc python tools/token_producer_cost.py
run 180 tokk_8 python benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 4 --batches-per-window 8
run 180 tokk_16_p6 python benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 6 --batches-per-window 16
