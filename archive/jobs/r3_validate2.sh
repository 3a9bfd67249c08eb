# Round 3 checkpoint: full GPU suite + smoke on the current tree, then the driver configuration 5x with
# the conservative counter order (t0 first; enqueued counter before the closing synchronize).
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3 4 5; do
  run 120 y_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/y_drv_$i.json
done
run 300 y_default python bench.py --json-out gpurun_out/y_default.json
for d in 2 4 6; do
  run 300 dh_bf16_d$d python benchmarks/bench_idle_sweep.py --floor --depth $d --ratios 0.5,0.75,0.9,1.25,2.0 --json-out gpurun_out/dh_bf16_d$d.jsonl
done
run 300 dh_u8_d4 python benchmarks/bench_idle_sweep.py --floor --depth 4 --source-dtype uint8 --ratios 0.5,0.75,0.9,1.25,2.0 --json-out gpurun_out/dh_u8_d4.jsonl
