# Round 5, thirteenth box: ddl_amd.DataLoader vs torch.utils.data.DataLoader on one map-style Dataset on the
# final tree (3 / 6 / 12 workers within the box's 16-CPU share), and the multi-rank GPU tests with the
# death watch beating for its rank.
source tools/gpu_job.sh
unset DDL_BACKEND
run 500 multirank_tests python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
for w in 3 6 12; do
  run 240 ddl_w$w python benchmarks/bench_dataloader.py --impl ddl --workers $w --json-out gpurun_out/dataloader_cmp.jsonl
  run 240 torch_w$w python benchmarks/bench_dataloader.py --impl torch --workers $w --json-out gpurun_out/dataloader_cmp.jsonl
done
