source tools/gpu_job.sh
run 300 res_bf16 python benchmarks/bench_resident.py --steps 1000 --warmup 50
run 300 res_bf16_b1024 python benchmarks/bench_resident.py --steps 400 --warmup 20 --batch 1024 --depths 2
run 300 res_u8 python benchmarks/bench_resident.py --steps 1000 --warmup 50 --dtype uint8 --depths 2
