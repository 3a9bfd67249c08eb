source tools/gpu_job.sh
rm -rf gpurun_out/prof_tok
run 200 prof_tok rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_tok -o tok --output-format csv -- python3 benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 6 --batches-per-window 16
