# Free event ordered after a skipped window's exchange: GPU tests, then host-bound benches for cost.
source tools/gpu_job.sh
run 600 gpu_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_exchange_gpu.py tests/test_loader_gpu.py tests/test_tokens.py
run 300 pointwise python benchmarks/bench_pointwise.py
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --steps 2000 --warmup 50
run 300 bench_ex env DDL_BACKEND=nccl python bench.py --exchange 0.5
