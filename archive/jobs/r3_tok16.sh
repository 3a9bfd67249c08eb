# Round 3: device pack plan + uint16 token transport (kernel and loader tests), the floor-under-traffic
# idle experiment, and the token feed with int32 vs uint16 tokens on the wire.
source tools/gpu_job.sh
run 300 t_kern python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_tokens.py -m gpu
run 300 tok_i32 python benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0
run 300 tok_u16 python benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0 --token-dtype uint16
run 300 tr_bf16 python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9 --floor --floor-traffic --json-out gpurun_out/tr_bf16.jsonl
run 300 tr_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --ratios 0.5,0.75,0.9 --floor --floor-traffic --json-out gpurun_out/tr_u8.jsonl
run 300 kbench python benchmarks/kernels_bench.py
