#!/bin/bash
# Round 6, the final tree: whole GPU suite (every test on the option records), smoke, the driver's command x2,
# a rocprofv3 kernel-trace summary of the driver's command (producers as threads under the profiler), config 5
# at N = 1 and config 4 on the final tree.
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 400 rocprof env DDL_PRODUCER_MODE=thread rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --json-out gpurun_out/bench_prof.json
run 200 res_n1 python benchmarks/bench_resident.py --steps 200 --warmup 20 --depths 1,2,4 --n-samples 32768
run 250 tokens python benchmarks/bench_tokens.py --batch 2048 --steps 2000 --warmup 100 --idle-steps 0 --token-dtype uint16
