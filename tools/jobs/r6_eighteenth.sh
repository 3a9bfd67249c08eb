#!/bin/bash
# Round 6: AQL queues in device memory (HSA_ALLOCATE_QUEUE_DEV_MEM=1) vs the default host-memory queues, on
# the driver's command: does the zero-copy path's per-step gap (27 us at every boundary) come from the command
# processor fetching packets over a link the gather saturates?
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2; do
  run 200 dev_$i env HSA_ALLOCATE_QUEUE_DEV_MEM=1 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/dev_$i.json
  run 200 host_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/host_$i.json
done
