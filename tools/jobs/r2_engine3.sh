source tools/gpu_job.sh
run 120 api_costs python -c "import json; from ddl_amd import _native; print(json.dumps(_native.hip().api_costs()))"
run 400 engine_tests python -u -m pytest tests/test_loader_gpu.py tests/test_checkpoint.py tests/test_kernels_gpu.py tests/test_tokens.py -m gpu -q -x --timeout 120 --timeout-method thread
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_native python benchmarks/bench_pointwise.py --dispatch native
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --idle-steps 0
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --idle-steps 0
