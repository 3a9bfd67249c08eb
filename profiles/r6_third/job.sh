#!/bin/bash
# Round 6, third box: the whole GPU suite on the refactored tree (option records, quarantine, replicated
# resident, dist block), smoke, the driver's N=1 line twice, and the N=8 on-card rehearsal over 200 windows
# for the exchange issue-wait p99.
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
export DDL_REHEARSAL=1 DDL_BACKEND=gloo
run 400 n8 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 8 --master-port 29671 bench.py --gpus 8 --steps 200 --warmup 5 --order window --pressure-ratio 0 --idle-steps 0 --json-out gpurun_out/n8.json
