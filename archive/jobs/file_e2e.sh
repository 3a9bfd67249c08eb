# End-to-end file-backed feed (uint8 file -> pread producers -> H2D -> normalised bf16) + idle behind PatchMLP.
source tools/gpu_job.sh
df -h "$TMPDIR" > gpurun_out/e2e_df.txt 2>&1
run 300 e2e_p4 python benchmarks/bench_file_e2e.py --producers 4 --keep
run 300 e2e_p8 python benchmarks/bench_file_e2e.py --producers 8 --keep
run 300 e2e_direct python benchmarks/bench_file_e2e.py --producers 8 --direct
