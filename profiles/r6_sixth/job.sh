#!/bin/bash
# Round 6, sixth box: the deep-tile zero-copy gather (16 accesses in flight per lane): zero-copy GPU tests, the
# kernel benchmark (no regression of the device gathers), and the zero-copy path under loader pressure at
# 4 / 8 / 16 / 32 workgroups.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 zc_tests python -u -m pytest tests/test_zerocopy.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread
for b in 4 8 16 32; do
  run 200 zc_$b python bench.py --steps 20 --warmup 5 --idle-steps 0 --zc-blocks $b --json-out gpurun_out/zc_$b.json
done
