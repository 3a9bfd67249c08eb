# Round 5, twenty-fifth box: the indexed phase with the headline's accounting (the smaller of the delivered
# rate and the device-timed landed bytes in the region): the driver's command x3, and the multi-rank bench
# GPU tests (torchrun and self-launch at N = 2).
source tools/gpu_job.sh
unset DDL_BACKEND
for i in 1 2 3; do
  run 200 bench_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/acct_$i.json
done
run 400 bench_tests python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu -k bench
