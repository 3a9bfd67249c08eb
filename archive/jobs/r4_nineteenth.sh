# Round 4, nineteenth box: direct-DMA staging (window copies straight onto SDMA engines through ROCr; no AQL
# packet waits on a copy). Correctness first (bit-identical batches vs HIP copy streams), then the idle at
# r = 0.9 / 0.95 and the feed (r = 1.25 point) vs the HIP-stream default, two and one engines.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 direct_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "direct_dma or copy_streams" -m gpu
SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95,1.25 --floor --steps 400 --feed-steps 200 --lead-diag"
run 200 host_1 $SW --json-out gpurun_out/host_1.jsonl
run 200 dma_1 $SW --direct-dma --json-out gpurun_out/dma_1.jsonl
run 200 dma1e_1 env DDL_COPY_STREAMS=1 $SW --direct-dma --json-out gpurun_out/dma1e_1.jsonl
run 200 host_2 $SW --json-out gpurun_out/host_2.jsonl
run 200 dma_2 $SW --direct-dma --json-out gpurun_out/dma_2.jsonl
run 200 dma1e_2 env DDL_COPY_STREAMS=1 $SW --direct-dma --json-out gpurun_out/dma1e_2.jsonl
