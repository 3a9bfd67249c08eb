# N>1 stream layout (exchange post-copy stream + RCCL + DDP streams) at 4 vs 8 hardware queues, 1-rank RCCL group.
source tools/gpu_job.sh
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" | tee gpurun_out/hwq_env.txt
for i in 1 2; do
run 300 hwq4_$i env GPU_MAX_HW_QUEUES=4 DDL_BACKEND=nccl python bench.py --exchange 0.5 --steps 200 --idle-steps 200
run 300 hwq8_$i env GPU_MAX_HW_QUEUES=8 DDL_BACKEND=nccl python bench.py --exchange 0.5 --steps 200 --idle-steps 200
done
