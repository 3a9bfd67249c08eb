# Round 5, twenty-sixth box: the whole GPU suite once more on the final tree (flakiness check before the
# driver's round-end run), then smoke.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
