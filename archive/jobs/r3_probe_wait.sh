source tools/gpu_job.sh
run 120 probe_a python benchmarks/probe_stream_wait.py
run 120 probe_b python benchmarks/probe_stream_wait.py --gemms 11 --m 8192 --iters 100
run 300 hw_look env DDL_ENGINE_HOST_WAIT=1 python benchmarks/bench_idle_sweep.py --floor --ratios 0.5,0.75,0.9 --json-out gpurun_out/hw_look.jsonl
run 300 sw_look python benchmarks/bench_idle_sweep.py --floor --ratios 0.5,0.75,0.9 --json-out gpurun_out/sw_look.jsonl
