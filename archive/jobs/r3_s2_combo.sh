# Round 3, session 2: copy-policy tests, N=2/4 gloo-on-card bench, token bench (auto wire dtype), zero-copy gather streams.
# the N > 1 path with the auto copy policy and pro-rata accounting.
source tools/gpu_job.sh
run 300 t_policy python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_loader_gpu.py -m gpu -k "copy_stream_policies or copy_policy_rejects"
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 300 s2_g2 $TR --nproc-per-node 2 --master-port 29641 bench.py --gpus 2 --steps 40 --warmup 10 --json-out gpurun_out/s2_g2.json
run 300 s2_g4 $TR --nproc-per-node 4 --master-port 29642 bench.py --gpus 4 --steps 40 --warmup 10 --json-out gpurun_out/s2_g4.json
run 300 s2_g2_self python bench.py --gpus 2 --steps 40 --warmup 10 --json-out gpurun_out/s2_g2_self.json
unset DDL_BACKEND
run 300 tok_auto python benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 200
run 200 t_zc python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_zerocopy.py -m gpu
run 200 zc_bf16 python benchmarks/bench_zerocopy.py --blocks 8,16,32,64 --prep-streams 1,2 --train-steps 0 --steps 300
run 200 zc_u8 python benchmarks/bench_zerocopy.py --dtype uint8 --blocks 32,64,0 --prep-streams 1,2 --train-steps 0 --steps 300
