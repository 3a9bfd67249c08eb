# Host-path breakdown of the token consumer (config 4): cProfile of the consumer process.
source tools/gpu_job.sh
run 300 tok_cprof python -m cProfile -s tottime benchmarks/bench_tokens.py --steps 3000 --mode pack
