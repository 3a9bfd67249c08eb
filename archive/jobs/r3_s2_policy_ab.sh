# Round 3, session 2: copy-stream policy A/B on the headline (200 steps, interleaved), pro-rata accounting.
source tools/gpu_job.sh
for i in 1 2 3; do
  run 200 ab_adaptive_$i python bench.py --order window --idle-steps 0 --json-out gpurun_out/ab_adaptive_$i.json
  run 200 ab_alternate_$i env DDL_COPY_POLICY=alternate python bench.py --order window --idle-steps 0 --json-out gpurun_out/ab_alternate_$i.json
  run 200 ab_one_$i env DDL_COPY_STREAMS=1 python bench.py --order window --idle-steps 0 --json-out gpurun_out/ab_one_$i.json
done
run 200 h2d_probe python benchmarks/probe_h2d.py
