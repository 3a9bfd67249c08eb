# Round 4, twelfth box: run-ahead events back to one per max_ahead/4 batches (PatchMLP idle), the pressure
# phase's multiplicative step correction (ratio must land at 0.9 +- 0.03); driver bench x3.
source tools/gpu_job.sh
unset DDL_BACKEND
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_c.json
