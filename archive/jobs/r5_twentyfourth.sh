# Round 5, twenty-fourth box: the indexed phase's ratio to the headline with and without the idle phases
# before it (the driver's command vs --idle-steps 0 --pressure-ratio 0), interleaved.
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2 3; do
  run 200 full_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/idx_full_$i.json
  run 200 bare_$i python bench.py --steps 20 --warmup 5 --idle-steps 0 --pressure-ratio 0 --json-out gpurun_out/idx_bare_$i.json
done
