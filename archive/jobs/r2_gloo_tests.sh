source tools/gpu_job.sh
run 600 mr_tests python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 240 --timeout-method thread
export DDL_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run 200 gloo_tok_n2 $TR --nproc-per-node 2 --master-port 29631 benchmarks/bench_tokens.py --steps 300 --warmup 30
run 200 gloo_res_n2 $TR --nproc-per-node 2 --master-port 29632 benchmarks/bench_resident.py --steps 100 --warmup 10 --depths 2
