# ZeroCopyLoader default grid cap by dtype (32 for same-width copies, uncapped for uint8 -> bf16).
source tools/gpu_job.sh
run 300 zc_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_zerocopy.py -m gpu
run 300 bench_a python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 300 bench_b python bench.py --json-out gpurun_out/bench_b.json
run 300 bench_u8 python bench.py --source-dtype uint8 --json-out gpurun_out/bench_u8.json
