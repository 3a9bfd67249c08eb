#!/bin/bash
# Round 6, first box: the self-verifying dist block (1-rank RCCL), the device-sharing refusal, the on-card
# gloo rehearsals that now label themselves, and the driver's N=1 line with pressure idle on the
# world-size-invariant paths.
source tools/gpu_job.sh
unset DDL_BACKEND
run 30 box_env bash -c 'env | grep -i -E "visible|gpu_max|hsa_" ; ls /dev/dri | head; nproc'
run 600 gpu_new python -u -m pytest tests/test_bench_gpu.py tests/test_multirank_gpu.py -q -x -v --timeout 240 --timeout-method thread
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
