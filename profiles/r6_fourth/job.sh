#!/bin/bash
# Round 6, fourth box: the whole GPU suite again (the free-event close test puts its spin in front of the
# window's last batch kernel; zero-copy hand-off modes), then the zero-copy gather under loader pressure:
# host vs device hand-off, and its workgroup count.
source tools/gpu_job.sh
unset DDL_BACKEND
run 1000 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 200 zc_device python bench.py --steps 20 --warmup 5 --idle-steps 0 --zc-handoff device --json-out gpurun_out/zc_device.json
run 200 zc_host python bench.py --steps 20 --warmup 5 --idle-steps 0 --zc-handoff host --json-out gpurun_out/zc_host.json
for b in 16 64; do
  run 200 zc_host_$b python bench.py --steps 20 --warmup 5 --idle-steps 0 --zc-blocks $b --json-out gpurun_out/zc_host_$b.json
done
