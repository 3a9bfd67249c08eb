# Round 5, fifteenth box: the whole GPU suite, smoke and the driver's command after the front-end session,
# torch-signature DataLoader and death-watch heartbeat changes.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
