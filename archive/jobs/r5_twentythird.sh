# Round 5, twenty-third box: what sets the indexed phase's ratio to the headline in the driver's 20-step
# command -- the driver's command x3 against the same with 20 warmup steps x3, interleaved.
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2 3; do
  run 200 d_$i python bench.py --steps 20 --warmup 5 --idle-steps 0 --pressure-ratio 0 --json-out gpurun_out/idx_d_$i.json
  run 200 w_$i python bench.py --steps 20 --warmup 20 --idle-steps 0 --pressure-ratio 0 --json-out gpurun_out/idx_w_$i.json
done
