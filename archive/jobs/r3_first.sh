# Round 3, first GPU pass: the new live-restore + exchange-engine tests, the multirank (gloo on the card)
# checks of the exchange-on native dispatch, the driver-config bench and the full-refill variant.
source tools/gpu_job.sh
run 600 t_new python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_live_restore_gpu.py tests/test_exchange_gpu.py tests/test_checkpoint.py -m gpu
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 300 bench_full python bench.py --steps 100 --warmup 10 --idle-steps 0 --order window --refill full --json-out gpurun_out/bench_full.json
run 400 t_multi python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
