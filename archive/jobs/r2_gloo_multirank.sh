# Multi-rank GPU data path on the one-GPU box: RCCL refuses two ranks on one card
# (archive/profiles/r1_rccl_probe), so the DP group is gloo (DDL_BACKEND=gloo; its all-to-all on
# device tensors bounces through host memory). Every rank still runs the full device path:
# producers -> pinned shm -> H2D ring -> exchange -> gfx950 gather -> DDP train step.
source tools/gpu_job.sh
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 300 gloo_n2 $TR --nproc-per-node 2 --master-port 29621 bench.py --gpus 2 --steps 40 --warmup 10 --json-out gpurun_out/gloo_n2.json
run 300 gloo_n2_self python bench.py --gpus 2 --steps 40 --warmup 10 --json-out gpurun_out/gloo_n2_self.json
run 300 gloo_n4 $TR --nproc-per-node 4 --master-port 29622 bench.py --gpus 4 --steps 40 --warmup 10 --json-out gpurun_out/gloo_n4.json
run 300 gloo_n2_examples $TR --nproc-per-node 2 --master-port 29623 examples/run_ddl.py
