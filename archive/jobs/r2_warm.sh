source tools/gpu_job.sh
export DDL_HOST_LOG=1 DDL_STAGER_LOG=1
run 120 w_base python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/w_base.json
run 120 w_base2 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/w_base2.json
DDL_WARM_SDMA=0 run 120 w_off python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/w_off.json
run 120 w_long python bench.py --gpus 1 --order window --idle-steps 0 --json-out gpurun_out/w_long.json
run 120 w_inline python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --dispatch inline --json-out gpurun_out/w_inline.json
