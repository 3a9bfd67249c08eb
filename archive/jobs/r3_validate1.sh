# Round 3 validation of the new defaults: bench depth 4 + host hand-off (no exchange), strict
# enqueued-rate bound; idle sweeps (bf16, uint8, tokens with 6x4x2 producers).
source tools/gpu_job.sh
for i in 1 2 3 4 5; do
  run 120 x_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/x_drv_$i.json
done
run 300 x_sw_bf16 python benchmarks/bench_idle_sweep.py --floor --json-out gpurun_out/x_sw_bf16.jsonl
run 300 x_sw_u8 python benchmarks/bench_idle_sweep.py --floor --source-dtype uint8 --json-out gpurun_out/x_sw_u8.jsonl
run 300 x_sw_tok python benchmarks/bench_idle_sweep.py --floor --family tokens --json-out gpurun_out/x_sw_tok.jsonl
run 300 x_tok python benchmarks/bench_tokens.py --steps 300 --warmup 30
