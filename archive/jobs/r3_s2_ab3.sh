# Round 3, session 2: same-box A/B of the current auto policy vs strict alternation, driver configuration.
source tools/gpu_job.sh
for i in 1 2 3 4; do
  run 120 ab3_auto_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/ab3_auto_$i.json
  run 120 ab3_alt_$i env DDL_COPY_POLICY=alternate python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/ab3_alt_$i.json
done
