source tools/gpu_job.sh
run 900 gpu_tests python -m pytest tests -m gpu -q
run 300 kbench python benchmarks/kernels_bench.py
run 400 resident python benchmarks/bench_resident.py --depths 1,2,3
run 300 tokens python benchmarks/bench_tokens.py --mode pack
run 300 bench python bench.py
