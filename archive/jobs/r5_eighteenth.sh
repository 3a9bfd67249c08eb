# Round 5, eighteenth box: the kernel tests and the kernel benchmark after dropping the row-major
# RandomResizedCrop form, and the resident loader with augmentation x2.
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 kernel_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu
run 300 kbench python benchmarks/kernels_bench.py
run 300 res_u8_aug python benchmarks/bench_resident.py --dtype uint8 --augment
run 300 res_u8_aug2 python benchmarks/bench_resident.py --dtype uint8 --augment
