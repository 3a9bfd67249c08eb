source tools/gpu_job.sh
run 600 kernels python -m pytest tests/test_kernels_gpu.py -q
run 300 kbench python benchmarks/kernels_bench.py
