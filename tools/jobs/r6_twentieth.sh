#!/bin/bash
# Round 6: indexed loaders (zero-copy, HBM-resident) carve batches from blocks and record the caller's stream
# once per block instead of once per batch. Their GPU tests, the per-step gaps of the zero-copy path, and the
# driver's command x2 (zero-copy pressure idle in the JSON line).
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 gpu_tests python -u -m pytest tests/test_zerocopy.py tests/test_resident.py tests/test_multirank_gpu.py -m gpu -q -x --timeout 240 --timeout-method thread
run 120 zc32 python tools/pressure_gaps.py --path zero_copy --meter plain
run 120 zc32_b python tools/pressure_gaps.py --path zero_copy --meter plain
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 300 resident python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 1,2
run 300 resident_idle python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2 --idle-step-ms 1.25 --handoffs device,host
