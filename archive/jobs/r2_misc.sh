source tools/gpu_job.sh
run 240 resident python benchmarks/bench_resident.py
run 240 resident_u8_aug python benchmarks/bench_resident.py --dtype uint8 --augment
run 240 zerocopy python benchmarks/bench_zerocopy.py
run 300 file_e2e python benchmarks/bench_file_e2e.py
run 120 bench_u8 python bench.py --source-dtype uint8 --json-out gpurun_out/bench_u8.json
