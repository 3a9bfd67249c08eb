# Round 4, second box: GPU test suite, driver bench x3 (pressure idle with the re-measured feed, indexed phase
# with the page prefault), idle sweep at the new default depth, NT-store A/B (kernels, resident), socket DRAM
# probe with more threads, N=8 gloo-on-card bench with the indexed phase.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
run 200 bench_n1_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_n1_a.json
run 200 bench_n1_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_n1_b.json
run 200 bench_n1_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_n1_c.json
run 300 sweep_bf16 python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,1.25 --floor --json-out gpurun_out/sweep_bf16.jsonl
run 200 kernels python benchmarks/kernels_bench.py
run 200 resident_plain python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2
run 200 resident_nt python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2 --nt-stores
run 200 socket_dram_wide python benchmarks/probe_socket_dram.py --dma-threads 12 --refill-threads 16 --json-out gpurun_out/socket_dram_wide.json
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 400 n8_torchrun $TR --nproc-per-node 8 --master-port 29641 bench.py --gpus 8 --steps 20 --warmup 5 --json-out gpurun_out/n8_torchrun.json
run 300 n4_torchrun $TR --nproc-per-node 4 --master-port 29642 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/n4_torchrun.json
