source tools/gpu_job.sh
run 300 engine_tests python -u -m pytest tests/test_loader_gpu.py tests/test_checkpoint.py tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_native python benchmarks/bench_pointwise.py --dispatch native
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
