# ddl_amd.DataLoader vs torch.utils.data.DataLoader on one map-style Dataset (uint8 3x224x224 + label).
source tools/gpu_job.sh
run 300 map_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_map_dataset.py -m gpu
for w in 3 6 12; do
  run 240 ddl_w$w python benchmarks/bench_dataloader.py --impl ddl --workers $w --json-out gpurun_out/dataloader_cmp.jsonl
  run 240 torch_w$w python benchmarks/bench_dataloader.py --impl torch --workers $w --json-out gpurun_out/dataloader_cmp.jsonl
done
