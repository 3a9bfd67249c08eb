# Config 4 with GPU idle % behind a fixed-cost token train step (pack and pad).
source tools/gpu_job.sh
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --steps 2000 --warmup 50 --idle-steps 300
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --steps 2000 --warmup 50 --idle-steps 300
