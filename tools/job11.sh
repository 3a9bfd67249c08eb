source tools/gpu_job.sh
run 600 tests_zc python -m pytest tests/test_zerocopy.py tests/test_resident.py tests/test_kernels_gpu.py -q
