# Round 3, session 2: the auto copy-stream policy (one stream while the consumer is the bottleneck, alternation
# while the loader is): headline throughput and idle below the crossover.
source tools/gpu_job.sh
for i in 1 2 3; do
  run 120 au_drv_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/au_drv_$i.json
done
for i in 1 2; do
  run 200 au_200_$i python bench.py --order window --idle-steps 0 --json-out gpurun_out/au_200_$i.json
done
R="--ratios 0.5,0.75,0.9,1.1,1.5 --floor"
run 300 au_sw_bf16 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/au_sw_bf16.jsonl
run 300 au_sw_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/au_sw_u8.jsonl
