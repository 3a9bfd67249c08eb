# Resident loader with on-device RandomResizedCrop: tests, then an ImageNet-size uint8 shard with augment.
source tools/gpu_job.sh
run 400 aug_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_loader_gpu.py -k "random_resized or resident or augment"
run 300 res_aug_small python benchmarks/bench_resident.py --dtype uint8 --depths 2 --steps 500 --warmup 50 --augment
run 500 res_aug_imagenet python benchmarks/bench_resident.py --dtype uint8 --n-samples 1281167 --depths 2 --steps 1000 --warmup 50 --augment
