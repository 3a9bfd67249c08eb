source tools/gpu_job.sh
run 120 host_py python tools/host_python_cost.py
run 400 tok_tests python -u -m pytest tests/test_tokens.py tests/test_checkpoint.py -x -v --timeout 120 --timeout-method thread -m gpu
for k in 1 8; do
run 180 tokk_$k python benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 4 --batches-per-window $k
done
run 180 tokk_16_p6 python benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 6 --batches-per-window 16
run 180 tokk_8_pad python benchmarks/bench_tokens.py --steps 2000 --warmup 100 --idle-steps 0 --producers 4 --mode pad --batches-per-window 8
run 180 tokk_8_idle python benchmarks/bench_tokens.py --steps 1000 --warmup 100 --idle-steps 300 --producers 4 --batches-per-window 8
for w in 256 1024; do
run 120 win_$w python bench.py --gpus 1 --steps 20 --warmup 5 --window $w --order window --json-out gpurun_out/win_$w.json
done
