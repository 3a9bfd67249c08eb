# Round 4, twenty-sixth box: the token config (4) fell from 26.5-26.8G to 17.1G tokens/s on the final staging,
# and the resident config from 5.74M to 5.31M. Same box A/B: device-memory AQL queues off, HIP copy streams,
# device-side waits.
source tools/gpu_job.sh
unset DDL_BACKEND
TOK="benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0 --token-dtype uint16"
run 200 tok_def python $TOK
run 200 tok_q0 env HSA_ALLOCATE_QUEUE_DEV_MEM=0 python $TOK
run 200 tok_streams python benchmarks/ab_run.py --stream-copies -- $TOK
run 200 tok_old env HSA_ALLOCATE_QUEUE_DEV_MEM=0 python benchmarks/ab_run.py --stream-copies --device-ready-wait --device-free-wait -- $TOK
run 200 tok_def2 python $TOK
RES="benchmarks/bench_resident.py --steps 300 --warmup 30 --depths 2"
run 200 res_def python $RES
run 200 res_q0 env HSA_ALLOCATE_QUEUE_DEV_MEM=0 python $RES
run 200 res_def2 python $RES
run 200 res_q0b env HSA_ALLOCATE_QUEUE_DEV_MEM=0 python $RES
