source tools/gpu_job.sh
run 900 all_tests python -m pytest tests -q --deselect tests/test_sanitizers.py
