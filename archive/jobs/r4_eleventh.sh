# Round 4, eleventh box: strict alternation (the auto copy policy removed): loader GPU tests incl. the HWC
# engine recipe; idle at fixed 1.5 / 1.8 ms steps vs prefetch depth and run-ahead bound; the driver bench.
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 loader_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py tests/test_bench_gpu.py
S="python benchmarks/bench_idle_sweep.py --step-ms 1.5,1.8 --floor --steps 300 --feed-steps 200"
for i in 1 2; do
  run 200 d4_$i $S --json-out gpurun_out/d4_$i.jsonl
  run 200 d6_$i $S --depth 6 --json-out gpurun_out/d6_$i.jsonl
  run 200 d8_$i $S --depth 8 --json-out gpurun_out/d8_$i.jsonl
  run 200 a32_$i $S --max-ahead 32 --json-out gpurun_out/a32_$i.jsonl
done
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
