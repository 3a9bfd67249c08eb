# Round 4, twentieth box: why direct-DMA staging was refused on the nineteenth box (reason string), then its
# correctness test and the idle A/B if it runs.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 direct_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "direct_dma" -m gpu
if grep -q " passed" gpurun_out/direct_tests.log && ! grep -q "failed" gpurun_out/direct_tests.log; then
  SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95,1.25 --floor --steps 400 --feed-steps 200 --lead-diag"
  run 200 host_1 $SW --json-out gpurun_out/host_1.jsonl
  run 200 dma_1 $SW --direct-dma --json-out gpurun_out/dma_1.jsonl
  run 200 dma1e_1 env DDL_COPY_STREAMS=1 $SW --direct-dma --json-out gpurun_out/dma1e_1.jsonl
  run 200 dma_2 $SW --direct-dma --json-out gpurun_out/dma_2.jsonl
  run 200 dma1e_2 env DDL_COPY_STREAMS=1 $SW --direct-dma --json-out gpurun_out/dma1e_2.jsonl
fi
