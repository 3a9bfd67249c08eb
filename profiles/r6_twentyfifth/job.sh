#!/bin/bash
# Round 6, the final tree: a rocprofv3 kernel-trace summary of the driver's command (producers as threads under
# the profiler, 100 steps).
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 rocprof env DDL_PRODUCER_MODE=thread rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --json-out gpurun_out/bench_prof.json
