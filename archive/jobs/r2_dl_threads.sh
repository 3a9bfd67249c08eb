source tools/gpu_job.sh
for w in 2 3 4; do for t in 1 2 4; do
  run 120 ddl_w${w}_t$t python benchmarks/bench_dataloader.py --impl ddl --workers $w --host-threads $t --json-out gpurun_out/dl_threads.jsonl
done; done
