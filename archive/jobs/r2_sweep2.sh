# Idle sweep re-run with the end-of-round defaults (two copy streams, whole-window dispatch, token windows k=1 here)
source tools/gpu_job.sh
run 300 sweep2_bf16 python benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep2_bf16.jsonl
run 300 sweep2_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --json-out gpurun_out/sweep2_u8.jsonl
run 300 sweep2_tok python benchmarks/bench_idle_sweep.py --family tokens --json-out gpurun_out/sweep2_tok.jsonl
