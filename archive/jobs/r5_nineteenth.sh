# Round 5, nineteenth box: same-box A/B of the resident loader with on-device augmentation, the column-major
# RandomResizedCrop (this tree) vs the row-major one (ab_old/: the tree before that change, built in place),
# interleaved.
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2; do
  run 300 res_aug_new_$i python benchmarks/bench_resident.py --dtype uint8 --augment --depths 2
  run 300 res_aug_old_$i env PYTHONPATH=$PWD/ab_old python ab_old/benchmarks/bench_resident.py --dtype uint8 --augment --depths 2
done
