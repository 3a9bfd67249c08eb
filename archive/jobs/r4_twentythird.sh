# Round 4, twenty-third box: what is left of the idle at r = 0.9 with direct DMA (~0.5 pp above the meter
# floor): run-ahead bound (events on the compute stream), gather grid cap, AQL queues in device memory,
# inline dispatch; two runs each at r = 0.9 / 0.95.
source tools/gpu_job.sh
unset DDL_BACKEND
SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95 --floor --steps 400 --feed-steps 200 --lead-diag"
for rep in 1 2; do
  run 200 def_$rep $SW --json-out gpurun_out/def_$rep.jsonl
  run 200 a8_$rep $SW --max-ahead 8 --json-out gpurun_out/a8_$rep.jsonl
  run 200 a32_$rep $SW --max-ahead 32 --json-out gpurun_out/a32_$rep.jsonl
  run 200 g64_$rep $SW --gather-blocks 64 --json-out gpurun_out/g64_$rep.jsonl
  run 200 qdev_$rep env HSA_ALLOCATE_QUEUE_DEV_MEM=1 $SW --json-out gpurun_out/qdev_$rep.jsonl
  run 200 inl_$rep $SW --dispatch inline --json-out gpurun_out/inl_$rep.jsonl
done
