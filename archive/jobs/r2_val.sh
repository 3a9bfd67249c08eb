source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 120 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 120 bench_default python bench.py --json-out gpurun_out/bench_default.json
run 120 bench_u8 python bench.py --source-dtype uint8 --json-out gpurun_out/bench_u8.json
run 300 host_cost python tools/loader_host_cost.py
run 200 pw_inline python benchmarks/bench_pointwise.py
run 200 tok_pack python benchmarks/bench_tokens.py --mode pack
run 200 tok_pad python benchmarks/bench_tokens.py --mode pad
run 200 kernels python benchmarks/kernels_bench.py
