# Round 5, twenty-second box: the multi-rank GPU tests, now with a rank SIGKILLed mid-epoch on the card
# (H2D copies, kernels and exchange collectives in flight).
source tools/gpu_job.sh
unset DDL_BACKEND
run 500 multirank_tests python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
