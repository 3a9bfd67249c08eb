# Round 3, session 2: device-timed pro-rata landed bytes (bench.py value), adaptive copy streams; full
# image sweeps with the tuned calibrated step; token sweep feed diagnosis (read ids vs all, keepalive).
source tools/gpu_job.sh
run 300 t_interval python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_loader_gpu.py -m gpu -k "interval or time_window or native_stager"
for i in 1 2 3 4 5; do
  run 120 pr_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/pr_drv_$i.json
done
run 200 pr_default python bench.py --json-out gpurun_out/pr_default.json
R="--floor"
run 400 sw_bf16 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/sw_bf16.jsonl
run 400 sw_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/sw_u8.jsonl
run 300 tok_bench python benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0
run 400 sw_tok_ids python benchmarks/bench_idle_sweep.py --family tokens --read ids $R --json-out gpurun_out/sw_tok_ids.jsonl
run 400 sw_tok_all python benchmarks/bench_idle_sweep.py --family tokens --read all $R --json-out gpurun_out/sw_tok_all.jsonl
