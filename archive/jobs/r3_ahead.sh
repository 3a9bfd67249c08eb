# Round 3: the run-ahead bound (max_ahead, default 16) vs none, and one vs two copy streams.
source tools/gpu_job.sh
R="--ratios 0.5,0.75,0.9,1.1,1.5 --floor"
run 200 ah16 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/ah16.jsonl
run 200 ah0 env DDL_MAX_AHEAD=0 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/ah0.jsonl
run 200 ah8 env DDL_MAX_AHEAD=8 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/ah8.jsonl
run 200 ah16_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/ah16_u8.jsonl
run 120 drv python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/drv_ah.json
