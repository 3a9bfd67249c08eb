source tools/gpu_job.sh
run 120 attr_p4_k8 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 4 --batches-per-window 8
run 120 attr_p6_k16 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --batches-per-window 16
run 120 attr_p6_k16_s2 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --slots 2 --batches-per-window 16
