# Round 5, eighth box: the driver's command x3 with the indexed phase on producers (spare producer set) and
# zero-copy; bench / multi-rank GPU tests (N = 2 on the card with the new phase).
source tools/gpu_job.sh
unset DDL_BACKEND
for i in a b c; do
  run 200 bench_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_$i.json
done
run 600 bench_tests python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_bench_gpu.py tests/test_multirank_gpu.py -m gpu
