# Round 3: idle below the crossover with the host hand-off at prefetch depth 2 / 4 / 6.
source tools/gpu_job.sh
for d in 2 4 6; do
  run 300 dh_bf16_d$d python benchmarks/bench_idle_sweep.py --floor --depth $d --ratios 0.5,0.75,0.9,1.25,2.0 --json-out gpurun_out/dh_bf16_d$d.jsonl
done
run 300 dh_u8_d4 python benchmarks/bench_idle_sweep.py --floor --depth 4 --source-dtype uint8 --ratios 0.5,0.75,0.9,1.25,2.0 --json-out gpurun_out/dh_u8_d4.jsonl
