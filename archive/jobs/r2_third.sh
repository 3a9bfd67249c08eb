# GPU tests after checkpoint/priority work; headline bench (window + indexed); idle sweeps; kernel roofline.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 300 bench_default python bench.py --json-out gpurun_out/bench_default.json
DDL_BATCH_STREAM_PRIORITY=normal run 300 sweep_bf16_normalprio python benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep_bf16_normalprio.jsonl
run 300 sweep_bf16 python benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep_bf16.jsonl
run 300 sweep_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --json-out gpurun_out/sweep_u8.jsonl
run 300 sweep_tok python benchmarks/bench_idle_sweep.py --family tokens --json-out gpurun_out/sweep_tok.jsonl
run 300 kernels python benchmarks/kernels_bench.py
