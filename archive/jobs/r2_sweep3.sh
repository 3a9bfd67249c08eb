source tools/gpu_job.sh
run 300 sweep3_tok python benchmarks/bench_idle_sweep.py --family tokens --json-out gpurun_out/sweep3_tok.jsonl
run 300 sweep3_bf16 python benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep3_bf16.jsonl
