# Round 5, twenty-first box: RandomResizedCrop variants interleaved on one box -- 2 adjacent columns per
# lane (this tree), 4 per lane (ab_k4/, same code with kCpl = 4), and the row-major form (ab_old/): kernel
# timings and the resident loader with augmentation. ab_k4's exactness: its own RRC tests.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 k4_tests env PYTHONPATH=$PWD/ab_k4 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -m gpu -k random_resized_crop
for t in new:. k4:ab_k4 old:ab_old; do
  n=${t%%:*}; d=${t#*:}
  run 120 kbench_$n env PYTHONPATH=$PWD/$d python $d/benchmarks/kernels_bench.py
done
for i in 1 2 3; do
  for t in new:. k4:ab_k4 old:ab_old; do
    n=${t%%:*}; d=${t#*:}
    run 300 res_aug_${n}_$i env PYTHONPATH=$PWD/$d python $d/benchmarks/bench_resident.py --dtype uint8 --augment --depths 2
  done
done
