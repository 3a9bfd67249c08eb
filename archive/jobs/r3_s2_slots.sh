# Round 3, session 2: producer slots 1 vs 2 in the driver configuration (interleaved): does a second slot per
# producer remove the link gaps left by a slow producer turnaround (one run at 91% link busy)?
source tools/gpu_job.sh
for i in 1 2 3 4 5 6; do
  run 120 sl1_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --slots 1 --json-out gpurun_out/sl1_$i.json
  run 120 sl2_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --slots 2 --json-out gpurun_out/sl2_$i.json
done
