# Round 4, eighteenth box: host-side copy waits are the default now (the engine waits for a window's copy on
# the host; the stager waits for a ring buffer's free event on the host; one marker per copy). GPU tests of
# the loader paths, the idle at r = 0.9 / 0.95 (default vs one copy stream vs the old device waits), and the
# driver's command (headline must hold).
source tools/gpu_job.sh
unset DDL_BACKEND
run 600 loader_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py tests/test_checkpoint.py tests/test_exchange_gpu.py tests/test_live_restore_gpu.py tests/test_verify_order.py -m gpu
SW="python benchmarks/bench_idle_sweep.py --ratios 0.9,0.95 --floor --steps 400 --feed-steps 200 --lead-diag"
run 200 host_1 $SW --json-out gpurun_out/host_1.jsonl
run 200 cs1_1 env DDL_COPY_STREAMS=1 $SW --json-out gpurun_out/cs1_1.jsonl
run 200 dev_1 $SW --device-ready-wait --device-free-wait --json-out gpurun_out/dev_1.jsonl
run 200 host_2 $SW --json-out gpurun_out/host_2.jsonl
run 200 cs1_2 env DDL_COPY_STREAMS=1 $SW --json-out gpurun_out/cs1_2.jsonl
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_cs1 env DDL_COPY_STREAMS=1 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_cs1.json
