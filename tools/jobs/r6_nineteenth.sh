#!/bin/bash
# Round 6: the zero-copy path's per-step gap (27 us at every boundary under the pressure step): with and without
# the allocator's cross-stream event per batch (record_stream), at 32 and 16 gather workgroups; the window path
# for reference.
source tools/gpu_job.sh
run 120 zc32 python tools/pressure_gaps.py --path zero_copy --meter plain
run 120 zc32_nors python tools/pressure_gaps.py --path zero_copy --meter plain --no-record-stream
run 120 zc16 python tools/pressure_gaps.py --path zero_copy --meter plain --zc-blocks 16
run 120 zc16_nors python tools/pressure_gaps.py --path zero_copy --meter plain --zc-blocks 16 --no-record-stream
run 120 win python tools/pressure_gaps.py --meter plain --copy-timing
# the driver's command with AQL queues in device memory vs the default (r6_eighteenth's runs, repeated here)
for i in 1 2; do
  run 200 qdev_$i env HSA_ALLOCATE_QUEUE_DEV_MEM=1 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/qdev_$i.json
  run 200 qhost_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/qhost_$i.json
done
