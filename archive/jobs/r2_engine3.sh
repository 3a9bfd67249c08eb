source tools/gpu_job.sh
run 120 api_costs python -c "import json; from ddl_amd import _native; print(json.dumps(_native.hip().api_costs()))"
run 400 engine_tests python -u -m pytest tests/test_loader_gpu.py tests/test_checkpoint.py tests/test_kernels_gpu.py tests/test_tokens.py -m gpu -q -x --timeout 120 --timeout-method thread
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_native python benchmarks/bench_pointwise.py --dispatch native
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --idle-steps 0
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --idle-steps 0
run 300 bench_default python bench.py --json-out gpurun_out/bench_default.json
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof_copy
run 400 rocprof_copy rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_copy -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 0 --order window
