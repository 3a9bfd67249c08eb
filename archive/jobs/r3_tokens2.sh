# Round 3: token feed with the corpus bound to the GPU's NUMA node (was wherever the creating thread ran).
source tools/gpu_job.sh
B="python benchmarks/bench_tokens.py --steps 300 --warmup 30 --idle-steps 0 --batch 2048 --n-seqs 65536"
for i in 1 2 3; do run 200 tn_b2k_$i $B; done
for i in 1 2; do run 200 tn_t4s2_$i $B --host-threads 4 --slots 2; done
for i in 1 2; do run 200 tn_p6t4s2_$i $B --host-threads 4 --slots 2 --producers 6; done
