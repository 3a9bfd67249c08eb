# Round 5, twenty-fifth box: the driver's command x3 after gc.freeze() before each timed region.
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2 3; do
  run 200 bench_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/gcf_$i.json
done
