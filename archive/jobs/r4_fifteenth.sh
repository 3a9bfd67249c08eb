# Round 4, fifteenth box: where the idle below the crossover sits (per-boundary gap distribution, host lead),
# at ratios tuned in the loop to 0.9 / 0.95, with the AQL queues in host (default) vs device memory.
source tools/gpu_job.sh
unset DDL_BACKEND
SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95 --floor --steps 400 --feed-steps 200 --lead-diag"
for rep in 1 2; do
  run 200 base_$rep $SW --json-out gpurun_out/base_$rep.jsonl
  run 200 qdev_$rep env HSA_ALLOCATE_QUEUE_DEV_MEM=1 $SW --json-out gpurun_out/qdev_$rep.jsonl
done
run 200 bench_base python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_base.json
run 200 bench_qdev env HSA_ALLOCATE_QUEUE_DEV_MEM=1 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_qdev.json
