# Round 5, first box: the changed GPU tests (bounded direct-DMA waits, bit-exact direct-DMA batches, exchange
# with a slow consumer, re-anchoring), the token config (4) after the O(n log n) FFD and streaming-store
# gathers (five runs), the driver's bench, and the exchange through a 1-rank RCCL group.
source tools/gpu_job.sh
unset DDL_BACKEND
run 600 gpu_tests python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_direct_dma_gpu.py tests/test_loader_gpu.py tests/test_exchange_gpu.py -m gpu
TOK="benchmarks/bench_tokens.py --batch 2048 --steps 2000 --warmup 100 --idle-steps 0 --token-dtype uint16"
for rep in 1 2 3 4 5; do
  run 150 tok_$rep python $TOK
done
run 200 bench python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench.json
run 200 exch_rccl env DDL_BACKEND=nccl python bench.py --steps 100 --warmup 10 --exchange 0.5 --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/exch_rccl.json
run 200 exch_none python bench.py --steps 100 --warmup 10 --exchange 0 --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/exch_none.json
