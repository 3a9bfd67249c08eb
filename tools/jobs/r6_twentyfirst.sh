#!/bin/bash
# Round 6, the final tree (block-carved indexed batches, drained pressure feed): whole GPU suite, smoke, the
# driver's command, the exchange through a 1-rank RCCL group, the N = 4 / 8 on-card rehearsals.
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 rccl1 env DDL_BACKEND=nccl python bench.py --steps 20 --warmup 5 --exchange 0.5 --json-out gpurun_out/rccl1.json
run 300 n4 env DDL_REHEARSAL=1 DDL_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4 --master-port 29693 bench.py --gpus 4 --steps 40 --warmup 5 --json-out gpurun_out/n4.json
run 400 n8 env DDL_REHEARSAL=1 DDL_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 8 --master-port 29694 bench.py --gpus 8 --steps 40 --warmup 5 --json-out gpurun_out/n8.json
