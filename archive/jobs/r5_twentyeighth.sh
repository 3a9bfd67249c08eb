# Round 5, twenty-eighth box: after adopting non-temporal gather loads -- the whole GPU suite, the driver's
# command x2, the resident loader (bf16, uint8, uint8 + augment) and the zero-copy loader bench.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 300 res_bf16 python benchmarks/bench_resident.py
run 300 res_u8 python benchmarks/bench_resident.py --dtype uint8
run 300 res_u8_aug python benchmarks/bench_resident.py --dtype uint8 --augment
run 120 kbench python benchmarks/kernels_bench.py
