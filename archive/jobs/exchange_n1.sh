# The global-shuffle exchange path (RCCL all-to-all on the post-copy stream) timed on one GPU:
# DDL_BACKEND=nccl builds a 1-rank RCCL group so bench.py runs the N>1 window pipeline at N=1.
source tools/gpu_job.sh
run 300 gpu_exchange_tests python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_exchange_gpu.py tests/test_loader_gpu.py
run 300 bench_noex python bench.py --steps 400 --warmup 40 --idle-steps 0 --json-out gpurun_out/bench_noex.json
run 300 bench_ex env DDL_BACKEND=nccl python bench.py --steps 400 --warmup 40 --idle-steps 0 --exchange 0.5 --json-out gpurun_out/bench_ex.json
run 300 bench_ex_sr env DDL_BACKEND=nccl python bench.py --steps 400 --warmup 40 --idle-steps 0 --exchange 0.5 --exchange-method sendrecv_replace --json-out gpurun_out/bench_ex_sr.json
