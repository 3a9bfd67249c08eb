#!/bin/bash
# Round 6: the N = 8 on-card rehearsal again (r6_twentyfirst's went 180 s without a line and was stopped; bench.py
# now prints a line per phase), and the N = 2 one.
source tools/gpu_job.sh
unset DDL_BACKEND
run 500 n8 env DDL_REHEARSAL=1 DDL_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 8 --master-port 29695 bench.py --gpus 8 --steps 40 --warmup 5 --json-out gpurun_out/n8.json
run 300 n2 env DDL_REHEARSAL=1 DDL_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 2 --master-port 29696 bench.py --gpus 2 --steps 40 --warmup 5 --json-out gpurun_out/n2.json
