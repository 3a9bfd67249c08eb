# Round 3: the driver configuration's 20-step spread comes from the copy engine restarting cold after
# the t0 barrier + synchronize (the ring is full, the stager parked). A deeper ring keeps it busy.
source tools/gpu_job.sh
for i in 1 2 3 4 5; do
  for d in 4 6 8; do
    run 120 w_d${d}_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --depth $d --json-out gpurun_out/w_d${d}_$i.json
  done
done
