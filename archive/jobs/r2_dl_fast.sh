source tools/gpu_job.sh
run 300 map_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_map_dataset.py tests/test_verify_order.py -m gpu
for w in 3 6; do
  run 240 ddl_w$w python benchmarks/bench_dataloader.py --impl ddl --workers $w --idle-steps 0 --json-out gpurun_out/dl_fast.jsonl
done
run 240 ddl_w3_t4 python benchmarks/bench_dataloader.py --impl ddl --workers 3 --host-threads 4 --idle-steps 0 --json-out gpurun_out/dl_fast.jsonl
run 240 torch_w6 python benchmarks/bench_dataloader.py --impl torch --workers 6 --idle-steps 0 --json-out gpurun_out/dl_fast.jsonl
