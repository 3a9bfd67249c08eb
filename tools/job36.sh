source tools/gpu_job.sh
run 900 gpu_tests python -m pytest tests -m gpu -q -x
