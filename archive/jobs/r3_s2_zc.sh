# Round 3, session 2: zero-copy gather with one vs two alternating gather streams (the link idles in a lone
# kernel's tail), correctness test, then the bench's indexed phase.
source tools/gpu_job.sh
run 200 t_zc python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_zerocopy.py -m gpu
run 200 zc_bf16 python benchmarks/bench_zerocopy.py --blocks 8,16,32,64 --prep-streams 1,2 --train-steps 0 --steps 300
run 200 zc_u8 python benchmarks/bench_zerocopy.py --dtype uint8 --blocks 32,64,0 --prep-streams 1,2 --train-steps 0 --steps 300
