# Config 5 at HBM scale: an ImageNet-size (1,281,167 x uint8 3x224x224 = 193 GB) shard resident in one
# MI355X's 288 GB HBM, and a 150 GB bf16 shard; exact global shuffle gather each step.
source tools/gpu_job.sh
{ free -g; df -h /dev/shm; } > gpurun_out/mem_before.txt 2>&1
run 500 res_u8_imagenet python benchmarks/bench_resident.py --dtype uint8 --n-samples 1281167 --depths 2 --steps 1000 --warmup 50
run 500 res_bf16_150g python benchmarks/bench_resident.py --dtype bfloat16 --n-samples 500000 --depths 1,2 --steps 1000 --warmup 50
