# Round 5, third box: what limits the zero-copy (indexed-order) gather -- load pattern, grid, streams
# (standalone probe and the loader's own sweep); the socket DRAM probe sized to the box's CPU share.
source tools/gpu_job.sh
unset DDL_BACKEND
run 60 cpu_share bash -c 'nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))"'
run 200 zc_probe benchmarks/bin/probe_zerocopy_read 4096
run 300 zc_sweep python benchmarks/bench_zerocopy.py --steps 600 --warmup 30 --blocks 16,24,32,48,64 --prep-streams 1,2 --train-steps 0
run 200 socket_nt_small python benchmarks/probe_socket_dram.py --dma-threads 4 --refill-threads 8 --stream-stores on --json-out gpurun_out/socket_nt_small.json
run 200 socket_plain_small python benchmarks/probe_socket_dram.py --dma-threads 4 --refill-threads 8 --stream-stores off --json-out gpurun_out/socket_plain_small.json
