# Round 5, thirtieth box: the other configs once more on the final tree -- tokens (config 4) x3, the uint8
# source normalised on the device x2, full-refill producers, the driver's command at N = 4 on the card over
# gloo, and ddl_amd.DataLoader vs torch's at 6 workers.
source tools/gpu_job.sh
unset DDL_BACKEND
TOK="benchmarks/bench_tokens.py --batch 2048 --steps 2000 --warmup 100 --idle-steps 0 --token-dtype uint16"
for i in 1 2 3; do
  run 250 tok_$i python $TOK
done
for i in 1 2; do
  run 200 u8_$i python bench.py --steps 100 --warmup 10 --source-dtype uint8 --idle-steps 0 --pressure-ratio 0 --order window --json-out gpurun_out/fin_u8_$i.json
done
run 250 refill python bench.py --refill full --steps 100 --warmup 10 --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/fin_refill.json
run 240 dl_ddl python benchmarks/bench_dataloader.py --impl ddl --workers 6 --json-out gpurun_out/fin_dataloader.jsonl
run 240 dl_torch python benchmarks/bench_dataloader.py --impl torch --workers 6 --json-out gpurun_out/fin_dataloader.jsonl
export DDL_BACKEND=gloo
run 300 n4 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4 --master-port 29652 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/fin_n4.json
