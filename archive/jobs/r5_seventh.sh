# Round 5, seventh box: why the wave-granular capped gather is fast in the probe (57.2 GB/s) but slow in the
# loader (174k): rocprofv3 kernel traces of the loader with each tiling, and interleaved plain runs.
source tools/gpu_job.sh
unset DDL_BACKEND
ZC="benchmarks/bench_zerocopy.py --steps 300 --warmup 20 --prep-streams 1 --train-steps 0"
for rep in 1 2; do
  run 200 zc_tile_$rep python $ZC --blocks 16,32
  run 200 zc_wave_$rep python $ZC --blocks 16,32 --capped-waves
done
run 300 prof_tile rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tile -o run -- python $ZC --blocks 32
run 300 prof_wave rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wave -o run -- python $ZC --blocks 32 --capped-waves
