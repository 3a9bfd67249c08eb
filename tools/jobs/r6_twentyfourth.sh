#!/bin/bash
# Round 6: 2 GB output blocks (batch engine and indexed loaders): whole GPU suite, smoke, the driver's command x2.
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 rccl1 env DDL_BACKEND=nccl python bench.py --steps 20 --warmup 5 --exchange 0.5 --json-out gpurun_out/rccl1.json
run 300 resident python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 1,2
