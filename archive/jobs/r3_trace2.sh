# Round 3: host-side markers (engine get, sweep get, output-block provides) under the idle-sweep trace,
# process-mode producers are not possible under rocprofv3 (threads), so also an untraced A/B.
source tools/gpu_job.sh
export DDL_PRODUCER_MODE=thread DDL_TRACE_ENGINE=1 DDL_SWEEP_MARKERS=1
rm -rf gpurun_out/trace_sweep2
run 400 trace_sweep2 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace_sweep2 -o sweep -- python3 benchmarks/bench_idle_sweep.py --ratios 0.5 --steps 60 --feed-steps 100 --json-out gpurun_out/sweep_traced2.jsonl
