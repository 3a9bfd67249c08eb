source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 bench python bench.py --json-out gpurun_out/bench.json
run 300 bench_u8 python bench.py --source-dtype uint8 --json-out gpurun_out/bench_u8.json
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof
run 400 rocprof rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30
