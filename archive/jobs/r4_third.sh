# Round 4, third box: the whole GPU suite, then A/B of the below-crossover idle at r = 0.9 (bf16): prefetch
# depth, run-ahead bound, batch-stream priority, dispatch mode, one copy stream.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu
S="python benchmarks/bench_idle_sweep.py --ratios 0.9 --floor --steps 300"
run 200 ab_default $S --json-out gpurun_out/ab_default.jsonl
run 200 ab_depth2 $S --depth 2 --json-out gpurun_out/ab_depth2.jsonl
run 200 ab_ahead0 $S --max-ahead 0 --json-out gpurun_out/ab_ahead0.jsonl
run 200 ab_prio_normal $S --batch-priority normal --json-out gpurun_out/ab_prio_normal.jsonl
run 200 ab_inline $S --dispatch inline --json-out gpurun_out/ab_inline.jsonl
DDL_COPY_STREAMS=1 run 200 ab_one_stream $S --json-out gpurun_out/ab_one_stream.jsonl
run 200 ab_default2 $S --json-out gpurun_out/ab_default2.jsonl
