#!/bin/bash
# Round 6: with the exchange on (1-rank RCCL group), the window's post-exchange ready event waited for on the
# batch stream (0, current) or on the host (1). Alternating, two runs each; then the exchange GPU tests.
source tools/gpu_job.sh
export DDL_BACKEND=nccl
for i in 1 2; do
  run 200 rdev_$i python bench.py --steps 100 --warmup 10 --exchange 0.5 --order window --idle-steps 0 --ready-event-host 0 --json-out gpurun_out/rdev_$i.json
  run 200 rhost_$i python bench.py --steps 100 --warmup 10 --exchange 0.5 --order window --idle-steps 0 --ready-event-host 1 --json-out gpurun_out/rhost_$i.json
done
