# Round 4, eighth box: one copy stream vs alternation at the SAME absolute step times (a ratio to each
# variant's own feed compared them at different step times), three interleaved runs each.
source tools/gpu_job.sh
unset DDL_BACKEND
S="python benchmarks/bench_idle_sweep.py --step-ms 1.55,1.7,2.0,2.8 --floor --steps 300 --feed-steps 200"
for i in 1 2 3; do
  run 200 alt_$i $S --copy-policy alternate --json-out gpurun_out/alt_$i.jsonl
  DDL_COPY_STREAMS=1 run 200 one_$i $S --json-out gpurun_out/one_$i.jsonl
done
