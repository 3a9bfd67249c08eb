source tools/gpu_job.sh
run 300 ktests python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "split or pack"
run 300 kbench python benchmarks/kernels_bench.py
run 120 pw_window python benchmarks/bench_pointwise.py --dispatch window
run 120 pw_inline python benchmarks/bench_pointwise.py --dispatch inline
run 120 pw_window_groups python benchmarks/bench_pointwise.py --dispatch window --consumer groups
