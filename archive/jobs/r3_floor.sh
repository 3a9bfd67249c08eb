# Round 3: the idle residual below the crossover does not move with prefetch depth; measure the
# meter's own floor (same step, held batch, no loader) and the dispatch variants.
source tools/gpu_job.sh
run 300 fl_look python benchmarks/bench_idle_sweep.py --floor --ratios 0.5,0.75,0.9 --json-out gpurun_out/fl_look.jsonl
run 300 fl_inline python benchmarks/bench_idle_sweep.py --floor --dispatch inline --ratios 0.5,0.75,0.9 --json-out gpurun_out/fl_inline.jsonl
run 300 fl_python python benchmarks/bench_idle_sweep.py --floor --dispatch python --ratios 0.5,0.75,0.9 --json-out gpurun_out/fl_python.jsonl
run 300 fl_u8 python benchmarks/bench_idle_sweep.py --floor --source-dtype uint8 --ratios 0.5,0.75,0.9 --json-out gpurun_out/fl_u8.jsonl
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/trace_floor
run 300 trace_floor rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace_floor -o sweep -- python3 benchmarks/bench_idle_sweep.py --floor --ratios 0.5 --steps 60 --feed-steps 100 --json-out gpurun_out/fl_traced.jsonl
unset DDL_PRODUCER_MODE
run 300 tok_k8 python benchmarks/bench_idle_sweep.py --family tokens --tokens-k 8 --floor --json-out gpurun_out/tok_k8.jsonl
