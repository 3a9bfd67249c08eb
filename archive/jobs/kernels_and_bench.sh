source tools/gpu_job.sh
run 600 gpu_kernel_tests python -m pytest tests/test_kernels_gpu.py -q -x
run 300 kernels python benchmarks/kernels_bench.py
run 300 bench python bench.py
