source tools/gpu_job.sh
run 400 ttests python -u -m pytest tests/test_tokens.py tests/test_loader_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu
run 120 tok_win_p6_k16 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --batches-per-window 16 --dispatch window
run 120 tok_inl_p6_k16 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --batches-per-window 16 --dispatch inline
run 120 tok_win_p4_k8 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 4 --batches-per-window 8
run 120 tok_win_pad python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --batches-per-window 16 --mode pad --dispatch window
run 200 host_cost env STEPS=3000 python tools/loader_host_cost.py
