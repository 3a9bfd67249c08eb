source tools/gpu_job.sh
run 600 gpu_tests python -m pytest tests -m gpu -q -x
run 200 probe python benchmarks/probe_h2d.py
export DDL_PRODUCER_MODE=thread
run 400 rocprof_mc rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof3 -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30
