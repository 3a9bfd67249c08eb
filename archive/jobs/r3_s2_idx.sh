# Round 3, session 2: why bench.py's indexed phase (177-180k) trails the standalone zero-copy bench (188k).
source tools/gpu_job.sh
run 200 ix_bench python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/ix_bench.json
run 200 ix_zc4096 python benchmarks/bench_zerocopy.py --n-samples 4096 --blocks 32 --train-steps 0 --steps 200
run 200 ix_zc16k python benchmarks/bench_zerocopy.py --n-samples 16384 --blocks 32 --train-steps 0 --steps 200
run 200 ix_numa python benchmarks/bench_numa.py
