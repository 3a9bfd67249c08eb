# Round 4, fifth box: is one copy stream below the crossover really better? Repeated sweeps at r = 0.75 and
# 0.9 under the auto policy (device-clock link-gap trigger), strict alternation and one copy stream, each
# point reporting how the copies ran (per stream, link busy, overlap, policy switches).
source tools/gpu_job.sh
unset DDL_BACKEND
S="python benchmarks/bench_idle_sweep.py --ratios 0.75,0.9 --floor --steps 300 --feed-steps 200"
for i in 1 2 3; do
  run 200 auto_$i $S --json-out gpurun_out/auto_$i.jsonl
  run 200 alt_$i $S --copy-policy alternate --json-out gpurun_out/alt_$i.jsonl
  DDL_COPY_STREAMS=1 run 200 one_$i $S --json-out gpurun_out/one_$i.jsonl
done
run 200 bench_x python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_x.json
