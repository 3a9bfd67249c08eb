source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 bench python bench.py --json-out gpurun_out/bench.json
