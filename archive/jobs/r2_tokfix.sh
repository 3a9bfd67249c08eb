source tools/gpu_job.sh
run 400 ttests python -u -m pytest tests/test_tokens.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu
for rep in 1 2; do
for tr in fixed exact; do
run 120 fx_${tr}_p6_k16_r$rep python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --batches-per-window 16 --token-rows $tr
run 120 fx_${tr}_p4_k8_r$rep python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 4 --batches-per-window 8 --token-rows $tr
done
done
