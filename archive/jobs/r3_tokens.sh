# Round 3: where the token feed (config 4) goes, and its run-to-run spread.
source tools/gpu_job.sh
B="python benchmarks/bench_tokens.py --steps 300 --warmup 30 --idle-steps 0"
run 200 tk_b64_1 $B
run 200 tk_b64_2 $B
run 200 tk_b2k_1 $B --batch 2048 --n-seqs 65536
run 200 tk_b2k_2 $B --batch 2048 --n-seqs 65536
run 200 tk_b2k_nopart env DDL_CPU_PARTITION=0 $B --batch 2048 --n-seqs 65536
run 200 tk_b2k_nopart2 env DDL_CPU_PARTITION=0 $B --batch 2048 --n-seqs 65536
run 200 tk_b2k_t4 $B --batch 2048 --n-seqs 65536 --host-threads 4
run 200 tk_b2k_p6 $B --batch 2048 --n-seqs 65536 --producers 6
