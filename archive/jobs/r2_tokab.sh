source tools/gpu_job.sh
for rep in 1 2; do
for cfg in "4 8" "6 16"; do
set -- $cfg
for d in window inline; do
run 120 ab_${d}_p$1_k$2_r$rep python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers $1 --batches-per-window $2 --dispatch $d
done
done
done
