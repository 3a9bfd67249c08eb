source tools/gpu_job.sh
run 600 gpu_tests python -u -m pytest tests/test_loader_gpu.py tests/test_tokens.py -x -v --timeout 120 --timeout-method thread -m gpu -k "native or held or window or token"
run 300 host_cost env STEPS=3000 python tools/loader_host_cost.py
run 120 pw_window python benchmarks/bench_pointwise.py --dispatch window
run 120 pw_window_groups python benchmarks/bench_pointwise.py --dispatch window --consumer groups
run 120 pw_inline python benchmarks/bench_pointwise.py --dispatch inline
