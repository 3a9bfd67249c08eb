source tools/gpu_job.sh
run 600 gpu_tests python -m pytest tests -m gpu -q
run 300 kernels python benchmarks/kernels_bench.py
run 300 bench python bench.py
