source tools/gpu_job.sh
run 900 gpu_tests python -m pytest tests -m gpu -q
run 300 tokens_pack python benchmarks/bench_tokens.py --mode pack
run 300 tokens_pad python benchmarks/bench_tokens.py --mode pad
run 400 resident_bf16 python benchmarks/bench_resident.py --depths 1,2,4
run 400 resident_u8 python benchmarks/bench_resident.py --dtype uint8 --depths 1,2
run 300 bench python bench.py
