# Round 3, session 2: auto copy policy with a run-length trigger (3 ring-waited windows in a row), interleaved
# with strict alternation: headline throughput (driver config and 200 steps) and idle below the crossover;
# plus the hipEventQuery probe.
source tools/gpu_job.sh
run 120 evq python benchmarks/probe_event_query.py
for i in 1 2 3; do
  run 120 a2_drv_auto_$i python bench.py --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/a2_drv_auto_$i.json
  run 120 a2_drv_alt_$i env DDL_COPY_POLICY=alternate python bench.py --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/a2_drv_alt_$i.json
done
for i in 1 2; do
  run 200 a2_200_auto_$i python bench.py --order window --idle-steps 0 --json-out gpurun_out/a2_200_auto_$i.json
  run 200 a2_200_alt_$i env DDL_COPY_POLICY=alternate python bench.py --order window --idle-steps 0 --json-out gpurun_out/a2_200_alt_$i.json
done
R="--ratios 0.5,0.75,0.9,1.1,1.5 --floor"
run 300 a2_sw_bf16 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/a2_sw_bf16.jsonl
run 300 a2_sw_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/a2_sw_u8.jsonl
