source tools/gpu_job.sh
for cfg in "2 8 2" "3 8 1" "3 8 2" "4 8 1" "3 16 1" "4 16 1" "2 16 2"; do
set -- $cfg
run 120 at_p$1_k$2_t$3 python benchmarks/bench_tokens.py --steps 3000 --warmup 200 --idle-steps 0 --producers $1 --batches-per-window $2 --host-threads $3
done
