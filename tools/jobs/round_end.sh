source tools/gpu_job.sh
run 900 gpu_tests python -m pytest tests -m gpu -q
run 300 bench python bench.py
run 300 bench_u8 python bench.py --source-dtype uint8
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof
run 400 rocprof rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30
