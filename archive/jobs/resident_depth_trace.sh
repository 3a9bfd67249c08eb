# Why depth 4 is slower than depth 1/2 on the resident loader: per-kernel times at each depth.
source tools/gpu_job.sh
for d in 2 4; do
  rm -rf gpurun_out/rd$d
  run 300 rd_trace_$d rocprofv3 --kernel-trace --stats -d gpurun_out/rd$d -o res --output-format csv -- python3 benchmarks/bench_resident.py --steps 1000 --warmup 50 --depths $d
done
