source tools/gpu_job.sh
for cfg in "4 1 8" "4 2 8" "6 1 8" "6 2 8" "8 2 8" "6 2 16" "8 1 16"; do
set -- $cfg
run 120 tok_p$1_s$2_k$3 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers $1 --slots $2 --batches-per-window $3
done
run 120 tok_pad_p6_s2_k16 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers 6 --slots 2 --batches-per-window 16 --mode pad
