source tools/gpu_job.sh
run 200 dbg_inline python tools/debug_inline.py
run 120 drv_a python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/drv_a.json
run 120 drv_b python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/drv_b.json
