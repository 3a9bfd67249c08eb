# Round 3: the below-crossover idle residual is the 2-deep ring (trace: the batch's copy lands late
# because the ring buffer it needs was freed just in time). Sweep the prefetch depth.
source tools/gpu_job.sh
for d in 2 3 4; do
  run 300 sweep_d$d python benchmarks/bench_idle_sweep.py --depth $d --ratios 0.5,0.75,0.9,1.25,2.0 --json-out gpurun_out/sweep_d$d.jsonl
done
for d in 2 3 4; do
  run 200 bench_d$d python bench.py --gpus 1 --steps 20 --warmup 5 --depth $d --json-out gpurun_out/bench_d$d.json
done
run 300 sweep_u8_d3 python benchmarks/bench_idle_sweep.py --depth 3 --source-dtype uint8 --ratios 0.5,0.75,0.9,1.25,2.0 --json-out gpurun_out/sweep_u8_d3.jsonl
run 300 sweep_tok_d3 python benchmarks/bench_idle_sweep.py --family tokens --depth 3 --json-out gpurun_out/sweep_tok_d3.jsonl
