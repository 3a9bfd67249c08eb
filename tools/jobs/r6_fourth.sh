#!/bin/bash
# Round 6, fourth box: the whole GPU suite again (the free-event close test now puts its spin in front of the
# window's last batch kernel), then the zero-copy gather's workgroup count under loader pressure.
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
for b in 16 64 128; do
  run 200 zc_$b python bench.py --steps 20 --warmup 5 --idle-steps 0 --zc-blocks $b --json-out gpurun_out/zc_$b.json
done
