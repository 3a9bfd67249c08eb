# Config 4 pack mode, in-order vs first-fit-decreasing rows (density), with GPU idle behind the token step.
source tools/gpu_job.sh
run 300 tok_gpu_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tokens.py
run 300 tok_ffd python benchmarks/bench_tokens.py --mode pack --pack-order ffd --steps 2000 --warmup 50 --idle-steps 300
run 300 tok_inorder python benchmarks/bench_tokens.py --mode pack --pack-order in_order --steps 2000 --warmup 50 --idle-steps 300
