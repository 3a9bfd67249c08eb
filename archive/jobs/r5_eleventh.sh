# Round 5, eleventh box: multi-rank GPU tests with the per-rank death watch (spawned before the GPU is
# touched), and the driver's command at N = 4 on the card over gloo.
source tools/gpu_job.sh
unset DDL_BACKEND
run 500 multirank_tests python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
export DDL_BACKEND=gloo
run 300 n4_torchrun python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4 --master-port 29642 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/n4_torchrun.json
