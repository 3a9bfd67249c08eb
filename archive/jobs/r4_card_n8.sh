# The driver's N=8 bench command on the one-GPU box: 8 rank processes share the card with the DP
# group on gloo (RCCL refuses two ranks on one GPU). Every rank runs its full device path:
# 3 producers -> pinned shm -> H2D ring -> all-to-all exchange -> gfx950 gather -> DDP train step,
# then the world-size-invariant indexed phase. Also configs 4 (tokens) and 5 (resident) at N=4/8.
source tools/gpu_job.sh
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 200 refetch_test python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_loader_gpu.py tests/test_bench_gpu.py -k "refetch or native_dispatch_matches or held_batches or pressure"
run 200 socket_dram python benchmarks/probe_socket_dram.py --json-out gpurun_out/socket_dram.json
run 200 hbm_ceilings benchmarks/bin/hbm_ceilings 4
run 200 bench_n1 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_n1.json
run 200 bench_full_refill python bench.py --refill full --steps 100 --warmup 10 --order window --idle-steps 0 --json-out gpurun_out/bench_full.json
run 400 n8_torchrun $TR --nproc-per-node 8 --master-port 29631 bench.py --gpus 8 --steps 20 --warmup 5 --json-out gpurun_out/n8_torchrun.json
run 400 n8_self python bench.py --gpus 8 --steps 20 --warmup 5 --json-out gpurun_out/n8_self.json
run 300 n4_torchrun $TR --nproc-per-node 4 --master-port 29632 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/n4_torchrun.json
run 300 tokens_n4 $TR --nproc-per-node 4 --master-port 29633 benchmarks/bench_tokens.py --steps 40 --warmup 10 --idle-steps 10
run 300 tokens_n8 $TR --nproc-per-node 8 --master-port 29634 benchmarks/bench_tokens.py --steps 40 --warmup 10 --idle-steps 10 --producers 3
run 300 resident_n4 $TR --nproc-per-node 4 --master-port 29635 benchmarks/bench_resident.py --steps 40 --warmup 10 --depths 2
run 300 resident_n8 $TR --nproc-per-node 8 --master-port 29636 benchmarks/bench_resident.py --steps 40 --warmup 10 --depths 2
run 300 indexed_probe_prefault python benchmarks/probe_indexed_phase.py
run 300 indexed_probe_noprefault python benchmarks/probe_indexed_phase.py --index-no-prefault
