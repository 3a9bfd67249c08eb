#!/bin/bash
# Round 6: the exchange-on path (every N > 1 run) through a 1-rank RCCL group: GPU idle at r = 0.9 with the
# engine handing lookahead batches off on the device (current) vs on the host. Alternating, two runs each.
source tools/gpu_job.sh
export DDL_BACKEND=nccl
for i in 1 2; do
  run 200 dev_$i python bench.py --steps 100 --warmup 10 --exchange 0.5 --order window --idle-steps 0 --exchange-handoff device --json-out gpurun_out/dev_$i.json
  run 200 host_$i python bench.py --steps 100 --warmup 10 --exchange 0.5 --order window --idle-steps 0 --exchange-handoff host --json-out gpurun_out/host_$i.json
done
