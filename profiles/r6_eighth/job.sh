#!/bin/bash
# Round 6: config 5 with an ImageNet-size uint8 dataset (1,281,167 x 3x224x224 = 193 GB) resident in one
# MI355X -- the replicated layout at N = 1, bring-up timed (load_s) -- and the bf16 depth sweep.
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 res_large python benchmarks/bench_resident.py --steps 400 --warmup 40 --depths 2 --dtype uint8 --n-samples 1281167
run 200 res_bf16 python benchmarks/bench_resident.py --steps 400 --warmup 40 --depths 1,2,4 --n-samples 65536
