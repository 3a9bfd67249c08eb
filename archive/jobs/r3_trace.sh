# Round 3: attribute the below-crossover idle residual (rocprofv3 kernel + copy + marker trace of the
# idle sweep at r = 0.5 / 0.75, producers as threads under the profiler), and the out-of-cache
# kernel rooflines (>= 1 GiB working sets).
source tools/gpu_job.sh
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/trace_sweep
run 400 trace_sweep rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace_sweep -o sweep -- python3 benchmarks/bench_idle_sweep.py --ratios 0.5,0.75 --steps 100 --json-out gpurun_out/sweep_traced.jsonl
unset DDL_PRODUCER_MODE
run 60 gaps0 python tools/trace_gaps.py gpurun_out/trace_sweep --range sweep.p00
run 60 gaps1 python tools/trace_gaps.py gpurun_out/trace_sweep --range sweep.p01
run 300 kernels python benchmarks/kernels_bench.py
rm -rf gpurun_out/trace_sweep/*/*kernel_trace.csv
