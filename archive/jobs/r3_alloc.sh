# Round 3: does the caching allocator growing new segments (hipMalloc) while the host runs ahead of the
# GPU cause the step-boundary gaps below the crossover? Same sweep without / with a pre-grown pool.
source tools/gpu_job.sh
run 200 al_0 python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9 --floor --json-out gpurun_out/al_0.jsonl
run 200 al_16 python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9 --floor --prealloc-gb 16 --json-out gpurun_out/al_16.jsonl
run 200 al_u8_16 python benchmarks/bench_idle_sweep.py --source-dtype uint8 --ratios 0.5,0.75,0.9 --floor --prealloc-gb 16 --json-out gpurun_out/al_u8_16.jsonl
