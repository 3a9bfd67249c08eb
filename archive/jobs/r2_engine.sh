# Native batch dispatch: GPU tests, host cost per batch, pointwise/image throughput (native vs python).
source tools/gpu_job.sh
run 300 engine_tests python -u -m pytest tests/test_loader_gpu.py tests/test_checkpoint.py -m gpu -q -x --timeout 120 --timeout-method thread
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_native python benchmarks/bench_pointwise.py --dispatch native
run 200 pw_python python benchmarks/bench_pointwise.py --dispatch python
run 200 pw_native_groups python benchmarks/bench_pointwise.py --dispatch native --consumer groups
run 300 bench_default python bench.py --json-out gpurun_out/bench_default.json
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
