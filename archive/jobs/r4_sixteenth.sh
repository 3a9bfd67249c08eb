# Round 4, sixteenth box: do the loader's streams share a hardware queue with the compute stream? HIP maps
# streams onto GPU_MAX_HW_QUEUES (default 4) AQL queues per priority; a stream that shares the compute
# stream's queue puts its barrier packets (waits on copies / gathers) in front of the step's kernels.
# A/B at ratios 0.9 / 0.95: 4 (default) vs 8 vs 16 queues; host-side copy waits (--ready-on-host).
source tools/gpu_job.sh
unset DDL_BACKEND
SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95 --floor --steps 400 --feed-steps 200 --lead-diag"
run 200 q4 $SW --json-out gpurun_out/q4.jsonl
run 200 q8 env GPU_MAX_HW_QUEUES=8 $SW --json-out gpurun_out/q8.jsonl
run 200 q16 env GPU_MAX_HW_QUEUES=16 $SW --json-out gpurun_out/q16.jsonl
run 200 roh $SW --ready-on-host --json-out gpurun_out/roh.jsonl
run 200 q16_roh env GPU_MAX_HW_QUEUES=16 $SW --ready-on-host --json-out gpurun_out/q16_roh.jsonl
run 200 q4b $SW --json-out gpurun_out/q4b.jsonl
run 200 q16b env GPU_MAX_HW_QUEUES=16 $SW --json-out gpurun_out/q16b.jsonl
run 200 bench_q16 env GPU_MAX_HW_QUEUES=16 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_q16.json
