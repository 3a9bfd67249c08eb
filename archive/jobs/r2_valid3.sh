source tools/gpu_job.sh
run 900 gpu_all python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 300 bench_default python bench.py --json-out gpurun_out/bench_default.json
