# Round 4, fourth box: the device-clock link-gap trigger of the auto copy policy. Idle sweep across the
# crossover, the driver bench x3 (headline must stay alternate-fast; pressure idle), copy-policy GPU tests,
# and the PCIe topology of the box.
source tools/gpu_job.sh
unset DDL_BACKEND
(lspci -tv > gpurun_out/lspci_tv.txt 2>&1 || true)
run 300 policy_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py tests/test_bench_gpu.py -k "copy or stager or pressure or refetch"
run 300 sweep python benchmarks/bench_idle_sweep.py --ratios 0.5,0.75,0.9,1.1,1.25 --floor --steps 300 --json-out gpurun_out/sweep_linkgap.jsonl
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 200 bench_c python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_c.json
run 200 bench_200 python bench.py --steps 200 --warmup 20 --json-out gpurun_out/bench_200.json
