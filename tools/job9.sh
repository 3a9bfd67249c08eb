source tools/gpu_job.sh
run 600 tests_zc python -m pytest tests/test_zerocopy.py tests/test_kernels_gpu.py tests/test_resident.py -q
run 400 zc_bf16 python benchmarks/bench_zerocopy.py
run 400 zc_u8 python benchmarks/bench_zerocopy.py --dtype uint8 --train-steps 0
