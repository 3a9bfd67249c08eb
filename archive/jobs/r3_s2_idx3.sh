# Round 3, session 2: indexed phase, same box: bench.py vs the standalone probe vs bench_zerocopy.
source tools/gpu_job.sh
run 200 i3_bench python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/i3_bench.json
run 200 i3_probe python benchmarks/probe_indexed_phase.py
run 200 i3_zc python benchmarks/bench_zerocopy.py --n-samples 4096 --blocks 32 --train-steps 0 --steps 200
run 200 i3_bench2 python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/i3_bench2.json
