# Round 4, seventeenth box: barrier packets waiting on other queues' work. The batch kernel's device-side wait
# for its window's copy (--ready-on-host moves it to the host) and the copy's device-side wait for the ring
# buffer's free event (--free-on-host). Ratios 0.9 / 0.95, the default 4 hardware queues.
source tools/gpu_job.sh
unset DDL_BACKEND
SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95 --floor --steps 400 --feed-steps 200 --lead-diag"
run 200 base $SW --json-out gpurun_out/base.jsonl
run 200 roh_1 $SW --ready-on-host --json-out gpurun_out/roh_1.jsonl
run 200 rf_1 $SW --ready-on-host --free-on-host --json-out gpurun_out/rf_1.jsonl
run 200 foh $SW --free-on-host --json-out gpurun_out/foh.jsonl
run 200 roh_2 $SW --ready-on-host --json-out gpurun_out/roh_2.jsonl
run 200 rf_2 $SW --ready-on-host --free-on-host --json-out gpurun_out/rf_2.jsonl
run 200 rf_cs1 env DDL_COPY_STREAMS=1 $SW --ready-on-host --free-on-host --json-out gpurun_out/rf_cs1.jsonl
run 200 roh_cs1 env DDL_COPY_STREAMS=1 $SW --ready-on-host --json-out gpurun_out/roh_cs1.jsonl
run 200 rf_slow python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75 --floor --steps 300 --feed-steps 200 --ready-on-host --free-on-host --json-out gpurun_out/rf_slow.jsonl
run 200 base_slow python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75 --floor --steps 300 --feed-steps 200 --json-out gpurun_out/base_slow.jsonl
