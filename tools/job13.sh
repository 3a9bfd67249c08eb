source tools/gpu_job.sh
run 600 gpu_tests python -m pytest tests -m gpu -q
run 300 bench python bench.py
run 300 bench_nosh python bench.py --shuffle none --idle-steps 100
