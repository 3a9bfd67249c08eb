# Round 4, twelfth box: run-ahead events back to one per max_ahead/4 batches (PatchMLP idle), the pressure
# phase's multiplicative step correction (ratio must land at 0.9 +- 0.03); driver bench x3.
source tools/gpu_job.sh
unset DDL_BACKEND
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_c.json
run 200 lead python benchmarks/bench_idle_sweep.py --step-ms 1.5,1.8,2.6 --floor --steps 300 --feed-steps 200 --lead-diag --json-out gpurun_out/lead.jsonl
run 200 lead_inline python benchmarks/bench_idle_sweep.py --step-ms 1.5,1.8 --steps 300 --feed-steps 200 --lead-diag --dispatch inline --json-out gpurun_out/lead_inline.jsonl
