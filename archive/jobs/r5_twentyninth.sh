# Round 5, twenty-ninth box: config 5 with non-temporal gather loads -- the ImageNet-size uint8 shard (193 GB)
# resident in one MI355X, and the default-size bf16 / uint8 shards x3 at prefetch depth 1 / 2.
source tools/gpu_job.sh
unset DDL_BACKEND
run 500 res_u8_imagenet python benchmarks/bench_resident.py --dtype uint8 --n-samples 1281167 --depths 2 --steps 1000 --warmup 50
for i in 1 2 3; do
  run 300 res_bf16_$i python benchmarks/bench_resident.py --depths 1,2
  run 300 res_u8_$i python benchmarks/bench_resident.py --dtype uint8 --depths 1,2
done
