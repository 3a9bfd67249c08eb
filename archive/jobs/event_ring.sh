# After the event-ring / token-collate host-path work: GPU tests, host-cost probe, configs 1/2/4/5.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
run 120 host_overhead python tools/host_overhead.py
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --steps 2000 --warmup 50
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --steps 2000 --warmup 50
run 300 pointwise python benchmarks/bench_pointwise.py
run 300 bench python bench.py
run 300 resident python benchmarks/bench_resident.py --steps 1000 --warmup 50 --depths 1,2,4
