# Round 3: the full GPU suite, smoke and the driver bench on the final tree.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --durations 25
run 300 smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 120 drv python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/drv.json
