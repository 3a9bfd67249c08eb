# Round 5, fifth box: the wave-granular capped gather (move_rows_waves) for the zero-copy indexed order:
# kernel / zero-copy GPU tests, the loader's grid x stream sweep three times, the driver's command twice.
source tools/gpu_job.sh
unset DDL_BACKEND
run 600 kernel_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_zerocopy.py -m gpu
for rep in 1 2 3; do
  run 300 zc_sweep_$rep python benchmarks/bench_zerocopy.py --steps 600 --warmup 30 --blocks 16,24,32,48 --prep-streams 1,2 --train-steps 0
done
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
