# Window free event recorded on the batch stream (no compute-stream wait per window).
source tools/gpu_job.sh
run 600 gpu_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py tests/test_exchange_gpu.py
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --steps 2000 --warmup 50
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --steps 2000 --warmup 50
run 300 pointwise python benchmarks/bench_pointwise.py
run 300 bench python bench.py
