# Round 5, fourth box: the zero-copy gather's load pattern, grid and streams, interleaved with repeats
# (standalone probe, 7 rounds), and the loader's own grid / stream sweep three times.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 zc_probe benchmarks/bin/probe_zerocopy_read 4096 7
for rep in 1 2 3; do
  run 300 zc_sweep_$rep python benchmarks/bench_zerocopy.py --steps 600 --warmup 30 --blocks 16,24,32 --prep-streams 1,2 --train-steps 0
done
