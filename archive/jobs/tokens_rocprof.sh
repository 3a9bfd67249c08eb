# Kernel and H2D stats of the config-4 token path (pack with FFD order, and pad), thread producers.
source tools/gpu_job.sh
rm -rf gpurun_out/prof_tok_pack gpurun_out/prof_tok_pad
run 300 rocprof_tok_pack rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_tok_pack -o tok --output-format csv -- python3 benchmarks/bench_tokens.py --mode pack --pack-order ffd --steps 500 --warmup 20 --idle-steps 0
run 300 rocprof_tok_pad rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_tok_pad -o tok --output-format csv -- python3 benchmarks/bench_tokens.py --mode pad --steps 500 --warmup 20 --idle-steps 0
