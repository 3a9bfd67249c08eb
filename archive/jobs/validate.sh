source tools/gpu_job.sh
run 120 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 900 gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 300 bench python bench.py
