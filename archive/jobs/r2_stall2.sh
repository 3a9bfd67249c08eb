source tools/gpu_job.sh
export DDL_HOST_LOG=1 DDL_STAGER_LOG=1
run 120 s_base python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/s_base.json
run 120 s_base2 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --dispatch python --json-out gpurun_out/s_base2.json
