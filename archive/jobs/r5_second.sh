# Round 5, second box: streaming-store A/B (socket DRAM probe, full-refill bench), multi-rank GPU tests, and
# a per-row SDMA gather probe for the indexed order, the 4- and 8-rank device path over gloo on the one card (final direct-DMA tree).
source tools/gpu_job.sh
unset DDL_BACKEND
run 200 sdma_rowgather benchmarks/bin/probe_sdma_rowgather 256 4096 60
run 200 socket_nt python benchmarks/probe_socket_dram.py --dma-threads 12 --refill-threads 16 --stream-stores on --json-out gpurun_out/socket_nt.json
run 200 socket_plain python benchmarks/probe_socket_dram.py --dma-threads 12 --refill-threads 16 --stream-stores off --json-out gpurun_out/socket_plain.json
run 250 refill_nt python bench.py --refill full --steps 100 --warmup 10 --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/refill_nt.json
run 250 refill_plain env DDL_STREAM_STORES=0 python bench.py --refill full --steps 100 --warmup 10 --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/refill_plain.json
run 400 multirank_tests python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 300 n4_torchrun $TR --nproc-per-node 4 --master-port 29642 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/n4_torchrun.json
run 400 n8_torchrun $TR --nproc-per-node 8 --master-port 29641 bench.py --gpus 8 --steps 20 --warmup 5 --json-out gpurun_out/n8_torchrun.json
