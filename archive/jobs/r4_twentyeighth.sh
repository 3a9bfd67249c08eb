# Round 4, twenty-eighth box: direct DMA with the one-engine placement while the consumer is the bottleneck
# (a window whose ring buffer was not free yet stays on the previous copy's engine) vs always alternating.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "direct_dma or copy_streams" -m gpu
SW="python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,0.95,1.25 --floor --steps 400 --feed-steps 200 --lead-diag"
for rep in 1 2; do
  run 200 pol_$rep $SW --one-engine-when-full --json-out gpurun_out/pol_$rep.jsonl
  run 200 alt_$rep $SW --json-out gpurun_out/alt_$rep.jsonl
  run 200 bpol_$rep python benchmarks/ab_run.py --one-engine-when-full -- bench.py --steps 20 --warmup 5 --json-out gpurun_out/bpol_$rep.json
  run 200 balt_$rep python bench.py --steps 20 --warmup 5 --json-out gpurun_out/balt_$rep.json
done
