# Round 3: the driver configuration 5x with the strict in-region copy count (copies enqueued AND retired
# inside the timed region), plus the multi-rank (gloo on the card) bench tests that read its JSON.
source tools/gpu_job.sh
for i in 1 2 3 4 5; do
  run 120 z_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/z_drv_$i.json
done
run 400 z_multi python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multirank_gpu.py -m gpu
