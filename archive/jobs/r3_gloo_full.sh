# Round 3: 2 and 4 DP ranks sharing the card (gloo DP group: RCCL refuses a shared card) with the
# exchange on (native engine path) and producers that rewrite their whole window every round.
source tools/gpu_job.sh
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 300 g2_stamp $TR --nproc-per-node 2 --master-port 29631 bench.py --gpus 2 --steps 40 --warmup 10 --json-out gpurun_out/g2_stamp.json
run 300 g2_full $TR --nproc-per-node 2 --master-port 29632 bench.py --gpus 2 --steps 40 --warmup 10 --refill full --slots 2 --producer-threads 8 --json-out gpurun_out/g2_full.json
run 300 g4_stamp $TR --nproc-per-node 4 --master-port 29633 bench.py --gpus 4 --steps 40 --warmup 10 --json-out gpurun_out/g4_stamp.json
run 300 g4_full $TR --nproc-per-node 4 --master-port 29634 bench.py --gpus 4 --steps 40 --warmup 10 --refill full --slots 2 --producer-threads 8 --json-out gpurun_out/g4_full.json
unset DDL_BACKEND
run 300 n1_full_def python bench.py --steps 100 --warmup 10 --idle-steps 0 --order window --refill full --slots 2 --producer-threads 8 --json-out gpurun_out/n1_full.json
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof_r3
run 400 rocprof_r3 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_r3 -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30 --order window
