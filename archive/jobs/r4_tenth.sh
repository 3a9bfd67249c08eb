# Round 4, tenth box: the HWC collate in the native engine (GPU test vs the Python path), the pressure phase
# with re-timing until the ratio lands at 0.9, and a rocprofv3 trace of the idle at a fixed 1.5 ms step
# (producers as threads under the profiler) for tools/trace_gaps.py.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 dispatch_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "native_dispatch"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
export DDL_PRODUCER_MODE=thread
run 300 trace_sweep rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace -o sweep -- python3 benchmarks/bench_idle_sweep.py --step-ms 1.5,2.0 --steps 150 --feed-steps 100 --json-out gpurun_out/sweep_traced.jsonl
unset DDL_PRODUCER_MODE
S="python benchmarks/bench_idle_sweep.py --step-ms 1.5,1.7,2.0 --floor --steps 300 --feed-steps 200"
for i in 1 2; do
  run 200 g0_$i $S --json-out gpurun_out/g0_$i.jsonl
  run 200 g32_$i $S --gather-blocks 32 --json-out gpurun_out/g32_$i.jsonl
  run 200 g64_$i $S --gather-blocks 64 --json-out gpurun_out/g64_$i.jsonl
  run 200 g128_$i $S --gather-blocks 128 --json-out gpurun_out/g128_$i.jsonl
done
