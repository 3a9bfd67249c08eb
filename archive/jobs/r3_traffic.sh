# Round 3: is the idle left below the crossover the loader's hand-off, or the loader's device traffic?
# The floor loop (one held batch, no loader) with and without the loader's copies running beside it,
# next to the loader run, per ratio; then a kernel trace of the r = 0.5 point for the gap attribution.
source tools/gpu_job.sh
run 300 tr_bf16 python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9 --floor --floor-traffic --json-out gpurun_out/tr_bf16.jsonl
run 300 tr_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --ratios 0.5,0.75,0.9 --floor --floor-traffic --json-out gpurun_out/tr_u8.jsonl
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/trace_traffic
run 400 trace_traffic rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace_traffic -o sweep -- python3 benchmarks/bench_idle_sweep.py --ratios 0.5 --steps 60 --feed-steps 100 --floor --floor-traffic --json-out gpurun_out/tr_traced.jsonl
