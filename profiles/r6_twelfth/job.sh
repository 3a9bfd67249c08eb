#!/bin/bash
# Round 6: the HBM-resident loader behind a fixed-cost step (1.5 ms), batches handed off on the device vs on the
# host, twice each.
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2; do
  run 200 res_idle_$i python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2 --n-samples 32768 --idle-step-ms 1.5 --handoffs device,host
done
