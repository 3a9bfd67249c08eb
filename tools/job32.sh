source tools/gpu_job.sh
run 600 gpu_rrc python -m pytest tests/test_kernels_gpu.py -q -x -k "random_resized"
