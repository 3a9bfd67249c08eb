# Round 3, session 2: copy-stream policy A/B with device-timed link occupancy per region.
source tools/gpu_job.sh
for i in 1 2; do
  run 200 ab2_adaptive_$i python bench.py --order window --idle-steps 0 --json-out gpurun_out/ab2_adaptive_$i.json
  run 200 ab2_alternate_$i env DDL_COPY_POLICY=alternate python bench.py --order window --idle-steps 0 --json-out gpurun_out/ab2_alternate_$i.json
  run 200 ab2_drv_adaptive_$i python bench.py --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/ab2_drv_adaptive_$i.json
  run 200 ab2_drv_alternate_$i env DDL_COPY_POLICY=alternate python bench.py --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/ab2_drv_alternate_$i.json
done
