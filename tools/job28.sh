source tools/gpu_job.sh
run 900 gpu_tests python -m pytest tests -m gpu -q -x
run 300 bench python bench.py
run 300 pointwise python benchmarks/bench_pointwise.py
