# Round 5, fourteenth box: config 5 at HBM scale on the final tree -- an ImageNet-size uint8 shard
# (1,281,167 x 3x224x224 = 193 GB) resident in one MI355X, exact global shuffle + normalised bf16 every step;
# and the on-device RandomResizedCrop + flip variant.
source tools/gpu_job.sh
{ free -g; df -h /dev/shm; } > gpurun_out/mem_before.txt 2>&1
run 500 res_u8_imagenet python benchmarks/bench_resident.py --dtype uint8 --n-samples 1281167 --depths 2 --steps 1000 --warmup 50
run 300 res_u8_aug python benchmarks/bench_resident.py --dtype uint8 --augment
