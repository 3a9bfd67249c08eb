# Round 3, session 2: bench.py indexed phase vs process context (CPU partition, NUMA bind, producers).
source tools/gpu_job.sh
run 200 ix_default python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/ix_default.json
run 200 ix_nopart env DDL_CPU_PARTITION=0 python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/ix_nopart.json
run 200 ix_nobind env DDL_NUMA_BIND=0 python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/ix_nobind.json
run 200 ix_thread env DDL_PRODUCER_MODE=thread python bench.py --order window+indexed --idle-steps 0 --json-out gpurun_out/ix_thread.json
