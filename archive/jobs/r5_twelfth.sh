# Round 5, twelfth box: the torch-signature DataLoader front end on the GPU (a training and an evaluation
# loader of one session, the second created mid-run), and the multi-rank GPU tests with the death watch
# standing down on a clean or aborted exit.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 frontend_tests python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_map_dataset.py -m gpu
run 500 multirank_tests python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
