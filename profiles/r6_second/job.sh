#!/bin/bash
# Round 6, second box: quarantine + stream-fallback staging tests; config 5 replicated vs sharded on the card
# (N=1 RCCL-free, N=2 gloo rehearsal); the exchange's issue-point host wait at N=4 / 8 (gloo on the card).
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 dma_tests python -u -m pytest tests/test_direct_dma_gpu.py -q -x -v --timeout 120 --timeout-method thread
run 200 res_n1 python benchmarks/bench_resident.py --steps 200 --warmup 20 --depths 2 --n-samples 32768
export DDL_REHEARSAL=1 DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 300 res_n2_rep $TR --nproc-per-node 2 --master-port 29661 benchmarks/bench_resident.py --steps 50 --warmup 10 --depths 2 --n-samples 8192 --replicate true
run 300 res_n2_shard $TR --nproc-per-node 2 --master-port 29662 benchmarks/bench_resident.py --steps 50 --warmup 10 --depths 2 --n-samples 8192 --replicate false
run 300 n4 $TR --nproc-per-node 4 --master-port 29663 bench.py --gpus 4 --steps 40 --warmup 5 --order window --pressure-ratio 0 --json-out gpurun_out/n4.json
run 400 n8 $TR --nproc-per-node 8 --master-port 29664 bench.py --gpus 8 --steps 40 --warmup 5 --order window --pressure-ratio 0 --json-out gpurun_out/n8.json
