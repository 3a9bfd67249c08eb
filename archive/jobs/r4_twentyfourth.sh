# Round 4, twenty-fourth box: validation with device-memory AQL queues as the default (set at import):
# whole GPU suite, smoke, the driver's command x3, the sweep, N=4 on the card over gloo.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
for i in a b c; do
  run 200 bench_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_$i.json
done
run 300 sweep python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,0.95,1.25 --floor --steps 400 --feed-steps 200 --lead-diag --json-out gpurun_out/sweep.jsonl
export DDL_BACKEND=gloo
run 400 n4_torchrun python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4 --master-port 29642 bench.py --gpus 4 --steps 20 --warmup 5 --json-out gpurun_out/n4_torchrun.json
