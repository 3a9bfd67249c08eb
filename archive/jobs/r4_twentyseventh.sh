# Round 4, twenty-seventh box: final configuration (direct DMA, host-side waits, the runtime's host-memory AQL
# queues): the driver's command x3; the token config A/B (direct DMA + host waits vs HIP streams + device
# waits), three runs each, interleaved.
source tools/gpu_job.sh
unset DDL_BACKEND
for i in a b c; do
  run 200 bench_$i python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_$i.json
done
TOK="benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0 --token-dtype uint16"
for rep in 1 2 3; do
  run 200 tok_def_$rep python $TOK
  run 200 tok_old_$rep python benchmarks/ab_run.py --stream-copies --device-ready-wait --device-free-wait -- $TOK
  run 200 tok_sh_$rep python benchmarks/ab_run.py --stream-copies -- $TOK
done
run 200 res_def python benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2
