# Round 3: kernel + copy + marker trace of the r = 0.5 bf16 point with the host hand-off (default), its
# floor (held batch) and its floor under the loader's traffic, for tools/trace_gaps.py per range; plus
# the pack-plan graph-replay bench rows.
source tools/gpu_job.sh
run 120 kb2 python benchmarks/kernels_bench.py
export DDL_PRODUCER_MODE=thread DDL_TRACE_ENGINE=1 DDL_SWEEP_MARKERS=1
rm -rf gpurun_out/trace_hh
run 400 trace_hh rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace_hh -o sweep -- python3 benchmarks/bench_idle_sweep.py --ratios 0.5 --steps 60 --feed-steps 100 --floor --floor-traffic --json-out gpurun_out/tr_traced.jsonl
cd tools
for r in sweep.p00 sweep.floor00 sweep.traffic00; do
  python trace_gaps.py ../gpurun_out/trace_hh --range $r > ../gpurun_out/gaps_$r.json || true
done
