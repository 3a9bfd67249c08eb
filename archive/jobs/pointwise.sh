source tools/gpu_job.sh
run 300 pointwise python benchmarks/bench_pointwise.py
run 300 pointwise_p1 python benchmarks/bench_pointwise.py --producers 1
run 300 pointwise_hs python benchmarks/bench_pointwise.py --host-shuffle
