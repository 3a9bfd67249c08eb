#!/bin/bash
# Round 6, last box: whole GPU suite on the final tree, smoke, the driver's command, and the exchange through a
# 1-rank RCCL group with its dist block (backend nccl, RCCL version, bus ID, device-timed all-to-all).
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 rccl1 env DDL_BACKEND=nccl python bench.py --steps 100 --warmup 10 --exchange 0.5 --order window --json-out gpurun_out/rccl1.json
