#!/bin/bash
# Round 6: the pressure phase times the feed after draining the rings phase 2 filled (the step was sized
# against a feed read ~4% high). The driver's command x3, the exchange through a 1-rank RCCL group, bench tests.
source tools/gpu_job.sh
unset DDL_BACKEND
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_c.json
run 200 rccl1 env DDL_BACKEND=nccl python bench.py --steps 20 --warmup 5 --exchange 0.5 --json-out gpurun_out/rccl1.json
run 400 bench_tests python -u -m pytest tests/test_bench_gpu.py -q -x --timeout 240 --timeout-method thread
