# Round 4, sixth box: the per-engine gap trigger of the auto copy policy across the crossover (it must switch
# to one stream below it and stay alternating above it), the driver bench x3 and the copy-policy GPU tests.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 policy_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py tests/test_bench_gpu.py -k "copy or stager or pressure"
S="python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,1.1,1.25 --floor --steps 300 --feed-steps 200"
run 200 sweep_1 $S --json-out gpurun_out/sweep_1.jsonl
run 200 sweep_2 $S --json-out gpurun_out/sweep_2.jsonl
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_c.json
