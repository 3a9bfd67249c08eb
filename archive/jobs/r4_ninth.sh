# Round 4, ninth box: the wide-band copy-mode trigger (one stream at >= 0.3 ms mean engine wait, back below
# 50 us) must leave the loader-bound headline alone; pressure phase over 300 steps; sweep at fixed step times;
# gather grid-cap A/B (64 / 256 workgroups vs the whole GPU).
source tools/gpu_job.sh
unset DDL_BACKEND
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_c.json
S="python benchmarks/bench_idle_sweep.py --step-ms 1.45,1.55,1.7,2.0,2.8 --floor --steps 300 --feed-steps 200"
run 200 auto_1 $S --json-out gpurun_out/auto_1.jsonl
run 200 g64_1 $S --copy-policy alternate --gather-blocks 64 --json-out gpurun_out/g64_1.jsonl
run 200 g256_1 $S --copy-policy alternate --gather-blocks 256 --json-out gpurun_out/g256_1.jsonl
run 200 alt_1 $S --copy-policy alternate --json-out gpurun_out/alt_1.jsonl
run 200 auto_2 $S --json-out gpurun_out/auto_2.jsonl
