# Round 5, first box: token config (4) after the O(n log n) FFD and streaming-store gathers, five runs; the
# socket DRAM probe and the full-refill bench with streaming stores on / off.
source tools/gpu_job.sh
unset DDL_BACKEND
TOK="benchmarks/bench_tokens.py --batch 2048 --steps 2000 --warmup 100 --idle-steps 0 --token-dtype uint16"
for rep in 1 2 3 4 5; do
  run 200 tok_$rep python $TOK
done
run 200 socket_nt python benchmarks/probe_socket_dram.py --dma-threads 12 --refill-threads 16 --stream-stores on --json-out gpurun_out/socket_nt.json
run 200 socket_plain python benchmarks/probe_socket_dram.py --dma-threads 12 --refill-threads 16 --stream-stores off --json-out gpurun_out/socket_plain.json
run 250 refill_nt python bench.py --refill full --steps 100 --warmup 10 --idle-steps 0 --order window --json-out gpurun_out/refill_nt.json
run 250 refill_plain env DDL_STREAM_STORES=0 python bench.py --refill full --steps 100 --warmup 10 --idle-steps 0 --order window --json-out gpurun_out/refill_plain.json
