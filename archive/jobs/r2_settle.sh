source tools/gpu_job.sh
for i in 1 2 3; do
run 120 drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/drv_$i.json
done
run 300 stage_tests python -u -m pytest tests/test_loader_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu
