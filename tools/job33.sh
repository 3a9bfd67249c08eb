source tools/gpu_job.sh
run 600 gpu_aug python -m pytest tests/test_loader_gpu.py -q -x -k "augment"
