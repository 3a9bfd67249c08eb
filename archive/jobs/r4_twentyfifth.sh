# Round 4, twenty-fifth box: the other configurations on the final staging (direct DMA, device-memory
# queues): tokens (config 4, uint16 ids and auto), full-refill producers, uint8 source, HBM-resident shuffle.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 tokens python benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0 --token-dtype uint16
run 300 tokens_auto python benchmarks/bench_tokens.py --steps 300 --warmup 30 --idle-steps 0
run 200 full python bench.py --refill full --steps 100 --warmup 10 --order window --idle-steps 0 --json-out gpurun_out/bench_full.json
run 200 u8 python bench.py --source-dtype uint8 --steps 100 --warmup 10 --order window --idle-steps 0 --json-out gpurun_out/bench_u8.json
run 300 resident python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2
