# GPU idle % sweep (calibrated step across the feed rate): images bf16, images uint8, tokens; trace cross-check.
source tools/gpu_job.sh
run 300 sweep_bf16 python benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep_bf16.jsonl
run 300 sweep_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --json-out gpurun_out/sweep_u8.jsonl
run 300 sweep_tok python benchmarks/bench_idle_sweep.py --family tokens --json-out gpurun_out/sweep_tok.jsonl
run 300 kernels python benchmarks/kernels_bench.py
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/trace_sweep
run 400 trace_sweep rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/trace_sweep -o sweep -- python3 benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep_traced.jsonl
python tools/trace_idle.py gpurun_out/trace_sweep --names sweep.p00,sweep.p01,sweep.p02,sweep.p03,sweep.p04,sweep.p05,sweep.p06,sweep.p07 --out gpurun_out/trace_sweep_idle.json
rm -rf gpurun_out/trace_sweep
