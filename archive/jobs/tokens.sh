source tools/gpu_job.sh
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --steps 1000 --warmup 50
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --steps 1000 --warmup 50
run 300 tok_pack2 python benchmarks/bench_tokens.py --mode pack --steps 1000 --warmup 50
