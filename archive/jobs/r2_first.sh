source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 300 bench_default python bench.py --json-out gpurun_out/bench_default.json
run 300 bench_w1024 python bench.py --window 1024 --json-out gpurun_out/bench_w1024.json
DDL_BACKEND=nccl run 300 bench_x1 python bench.py --exchange 0.5 --steps 100 --json-out gpurun_out/bench_x1.json
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof
run 400 rocprof rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30
