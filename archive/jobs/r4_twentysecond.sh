# Round 4, twenty-second box: direct-DMA staging with the global-shuffle exchange too (the consumer waits for
# the copy on the host, then enqueues the all-to-all). Exchange / multi-rank GPU tests, then the driver's
# N=2 and N=4 commands on the one card over gloo (exchange on, every rank direct DMA).
source tools/gpu_job.sh
unset DDL_BACKEND
run 600 xtests python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_exchange_gpu.py tests/test_multirank_gpu.py tests/test_live_restore_gpu.py -m gpu
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 300 n2_torchrun $TR --nproc-per-node 2 --master-port 29643 bench.py --gpus 2 --steps 20 --warmup 5 --json-out gpurun_out/n2_torchrun.json
run 400 n4_torchrun $TR --nproc-per-node 4 --master-port 29642 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/n4_torchrun.json
