# Round 3, second pass: early ring-buffer hand-back in the native engine.
# Full GPU suite, driver-config bench (early release on / off A/B), idle sweeps (the below-crossover
# residual), the NUMA local/remote read bench and the full-refill producer variants.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 300 bench_driver_late env DDL_EARLY_RELEASE=0 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver_late.json
run 300 sweep_bf16 python benchmarks/bench_idle_sweep.py --json-out gpurun_out/sweep_bf16.jsonl
run 300 sweep_bf16_late env DDL_EARLY_RELEASE=0 python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9 --json-out gpurun_out/sweep_bf16_late.jsonl
run 300 sweep_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --json-out gpurun_out/sweep_u8.jsonl
run 300 numa python benchmarks/bench_numa.py
run 200 full_s1 python bench.py --steps 100 --warmup 10 --idle-steps 0 --order window --refill full --json-out gpurun_out/full_s1.json
run 200 full_s2 python bench.py --steps 100 --warmup 10 --idle-steps 0 --order window --refill full --slots 2 --json-out gpurun_out/full_s2.json
run 200 full_p4 python bench.py --steps 100 --warmup 10 --idle-steps 0 --order window --refill full --producers 4 --slots 2 --json-out gpurun_out/full_p4.json
run 200 full_t8 python bench.py --steps 100 --warmup 10 --idle-steps 0 --order window --refill full --slots 2 --producer-threads 8 --json-out gpurun_out/full_t8.json
