source tools/gpu_job.sh
run 300 host_overhead python tools/host_overhead.py
run 300 pointwise python benchmarks/bench_pointwise.py
