source tools/gpu_job.sh
export DDL_STAGER_LOG=1
run 120 drv_a python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/drv_a.json
run 120 drv_p6 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --producers 6 --json-out gpurun_out/drv_p6.json
run 120 drv_s2 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --slots 2 --json-out gpurun_out/drv_s2.json
run 120 drv_long python bench.py --gpus 1 --steps 200 --warmup 20 --order window --idle-steps 0 --json-out gpurun_out/drv_long.json
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_inline python benchmarks/bench_pointwise.py --dispatch inline
run 200 pw_lookahead python benchmarks/bench_pointwise.py --dispatch lookahead
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --idle-steps 0
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --idle-steps 0
run 400 engine_tests python -u -m pytest tests/test_loader_gpu.py tests/test_tokens.py tests/test_checkpoint.py -m gpu -q -x --timeout 120 --timeout-method thread
