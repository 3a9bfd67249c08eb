source tools/gpu_job.sh
run 200 dbg_inline python tools/debug_inline.py
export DDL_STAGER_LOG=1
run 120 drv_a python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/drv_a.json
run 120 drv_b python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/drv_b.json
run 120 drv_long python bench.py --gpus 1 --order window --idle-steps 0 --json-out gpurun_out/drv_long.json
unset DDL_STAGER_LOG
run 400 engine_tests python -u -m pytest tests/test_loader_gpu.py tests/test_tokens.py tests/test_checkpoint.py -m gpu -q -x --timeout 120 --timeout-method thread
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_inline python benchmarks/bench_pointwise.py --dispatch inline
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --idle-steps 0
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/short_256
run 300 short_256 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/short_256 -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --idle-steps 0 --order window --json-out gpurun_out/short_256.json
