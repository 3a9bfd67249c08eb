# Round 5, twentieth box: RandomResizedCrop with 2 adjacent columns per lane (4 B stores) vs the row-major
# form (ab_old/: the tree before the column-major change, built in place): bit-exact tests, kernel timings,
# and the resident loader with augmentation, interleaved on one box.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 rrc_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k random_resized_crop
run 120 kbench_new python benchmarks/kernels_bench.py
run 120 kbench_old env PYTHONPATH=$PWD/ab_old python ab_old/benchmarks/kernels_bench.py
for i in 1 2 3; do
  run 300 res_aug_new_$i python benchmarks/bench_resident.py --dtype uint8 --augment --depths 2
  run 300 res_aug_old_$i env PYTHONPATH=$PWD/ab_old python ab_old/benchmarks/bench_resident.py --dtype uint8 --augment --depths 2
done
