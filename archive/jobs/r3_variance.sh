# Round 3: run-to-run spread of the driver configuration (20 steps, 5 warmup) at prefetch depth 2 / 3,
# stream-wait vs host-wait hand-off, interleaved on one box.
source tools/gpu_job.sh
for i in 1 2 3 4 5; do
  run 120 v_d2_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --depth 2 --json-out gpurun_out/v_d2_$i.json
  run 120 v_d3_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --depth 3 --json-out gpurun_out/v_d3_$i.json
  run 120 v_d3h_$i env DDL_ENGINE_HOST_WAIT=1 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --depth 3 --json-out gpurun_out/v_d3h_$i.json
done
