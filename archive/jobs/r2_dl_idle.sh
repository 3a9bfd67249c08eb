# ddl_amd.DataLoader vs torch DataLoader: feed rate and GPU idle % behind the PatchMLP train step.
source tools/gpu_job.sh
for w in 3 6; do
  run 240 ddl_w$w python benchmarks/bench_dataloader.py --impl ddl --workers $w --idle-steps 100 --json-out gpurun_out/dl_idle.jsonl
  run 300 torch_w$w python benchmarks/bench_dataloader.py --impl torch --workers $w --idle-steps 100 --json-out gpurun_out/dl_idle.jsonl
done
