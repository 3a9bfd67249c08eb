# Round 5, the other BASELINE configs on the final tree: tokens (config 4) with the token train step's idle,
# the HBM-resident global shuffle (config 5), the uint8 source, and the idle sweep of the bf16 feed; first
# the direct-DMA tests, incl. a 20,000-window run.
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 direct_tests python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_direct_dma_gpu.py -m gpu
run 250 tokens_idle python benchmarks/bench_tokens.py --batch 2048 --steps 2000 --warmup 100 --idle-steps 300 --token-dtype uint16
run 250 resident python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 1,2,4
run 200 bench_u8 python bench.py --steps 100 --warmup 10 --source-dtype uint8 --idle-steps 0 --pressure-ratio 0 --order window --json-out gpurun_out/bench_u8.json
run 400 sweep python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,1.25 --floor --json-out gpurun_out/sweep.jsonl
for t in 4 8; do
  for rep in 1 2; do
    run 200 idx_t${t}_$rep python bench.py --steps 20 --warmup 5 --idle-steps 0 --pressure-ratio 0 --index-threads $t --json-out gpurun_out/idx_t${t}_$rep.json
  done
done
