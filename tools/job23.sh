source tools/gpu_job.sh
run 300 cprof python -m cProfile -s tottime benchmarks/bench_pointwise.py --steps 2000
