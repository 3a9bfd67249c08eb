source tools/gpu_job.sh
run 400 verify_tests python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_verify_order.py tests/test_map_dataset.py tests/test_checkpoint.py -m gpu
