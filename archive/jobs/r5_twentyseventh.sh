# Round 5, twenty-seventh box: non-temporal loads in the row gathers (ab_nt/: this tree with the gather
# kernels' source loads marked nontemporal) against plain loads, interleaved on one box: the kernel
# benchmark, the HBM-resident loader (bf16 and uint8 shards) and the driver's command.
source tools/gpu_job.sh
unset DDL_BACKEND
for t in plain:. nt:ab_nt; do
  n=${t%%:*}; d=${t#*:}
  run 120 kbench_$n env PYTHONPATH=$PWD/$d python $d/benchmarks/kernels_bench.py
done
for i in 1 2; do
  for t in plain:. nt:ab_nt; do
    n=${t%%:*}; d=${t#*:}
    run 300 res_bf16_${n}_$i env PYTHONPATH=$PWD/$d python $d/benchmarks/bench_resident.py --depths 2
    run 300 res_u8_${n}_$i env PYTHONPATH=$PWD/$d python $d/benchmarks/bench_resident.py --dtype uint8 --depths 2
  done
done
