# Round 3: hand-off of lookahead batches by a host wait on the batch event (DDL_ENGINE_HOST_WAIT=1)
# vs the device-side stream wait, across the whole sweep and in the driver bench.
source tools/gpu_job.sh
run 300 hw_all env DDL_ENGINE_HOST_WAIT=1 python benchmarks/bench_idle_sweep.py --floor --json-out gpurun_out/hw_all.jsonl
run 300 sw_all python benchmarks/bench_idle_sweep.py --floor --json-out gpurun_out/sw_all.jsonl
run 300 hw_u8 env DDL_ENGINE_HOST_WAIT=1 python benchmarks/bench_idle_sweep.py --floor --source-dtype uint8 --json-out gpurun_out/hw_u8.jsonl
run 200 bd_hw env DDL_ENGINE_HOST_WAIT=1 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bd_hw.json
run 200 bd_sw python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bd_sw.json
run 200 bd_hw200 env DDL_ENGINE_HOST_WAIT=1 python bench.py --order window --json-out gpurun_out/bd_hw200.json
run 200 bd_sw200 python bench.py --order window --json-out gpurun_out/bd_sw200.json
run 300 tok_k8_keep python benchmarks/bench_idle_sweep.py --family tokens --tokens-k 8 --floor --feed-keepalive --json-out gpurun_out/tok_k8_keep.jsonl
