# Trace-based GPU idle % cross-check of the bench (kernel + copy + roctx marker trace; no PMC).
source tools/gpu_job.sh
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/trace
run 400 trace rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace -o bench -- python3 bench.py --steps 100 --warmup 10 --idle-steps 100
python tools/trace_idle.py gpurun_out/trace --out gpurun_out/trace_idle.json
