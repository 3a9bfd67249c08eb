# File-backed e2e: producers x pread threads on the box's 16-CPU share (page cache).
source tools/gpu_job.sh
run 300 e2e_p2t8 python benchmarks/bench_file_e2e.py --producers 2 --host-threads 8 --keep --idle-steps 0
run 300 e2e_p4t4 python benchmarks/bench_file_e2e.py --producers 4 --host-threads 4 --keep --idle-steps 0
run 300 e2e_p3t4 python benchmarks/bench_file_e2e.py --producers 3 --host-threads 4 --keep --idle-steps 0
run 300 e2e_p4t4s3 python benchmarks/bench_file_e2e.py --producers 4 --host-threads 4 --slots 3 --keep --idle-steps 0
run 300 e2e_p6t2 python benchmarks/bench_file_e2e.py --producers 6 --host-threads 2 --keep --idle-steps 0
run 300 e2e_p4t8 python benchmarks/bench_file_e2e.py --producers 4 --host-threads 8 --idle-steps 0
