# Rehearse the N>1 bench path on the single-GPU box: 2 ranks share cuda:0 over RCCL (if RCCL allows it).
source tools/gpu_job.sh
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611"
timeout -k 10 90 $TR tools/rccl_same_gpu_probe.py > gpurun_out/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -n 20 gpurun_out/probe.log
[ $rc -eq 0 ] || exit $rc
run 240 bench_n2 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 100 --warmup 10
