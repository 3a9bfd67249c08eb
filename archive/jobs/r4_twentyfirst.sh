# Round 4, twenty-first box: direct-DMA staging is the default. Whole GPU suite, smoke, the driver's command
# x3, the idle sweep (default vs HIP copy streams), and a rocprofv3 kernel-trace summary of the driver's
# command (producers as threads under the profiler).
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
for i in a b c; do
  run 200 bench_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_$i.json
done
SW="python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,0.95,1.25 --floor --steps 400 --feed-steps 200 --lead-diag"
run 300 sweep_dma $SW --json-out gpurun_out/sweep_dma.jsonl
run 300 sweep_streams $SW --stream-copies --json-out gpurun_out/sweep_streams.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 400 rocprof env DDL_PRODUCER_MODE=thread rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --json-out gpurun_out/bench_prof.json
