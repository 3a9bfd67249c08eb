source tools/gpu_job.sh
run 120 probe_a python benchmarks/probe_stream_wait.py
run 120 probe_b python benchmarks/probe_stream_wait.py --gemms 11 --m 8192 --iters 100
run 120 probe_c python benchmarks/probe_stream_wait.py --gemms 1 --m 1024 --iters 500
