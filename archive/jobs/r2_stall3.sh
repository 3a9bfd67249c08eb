source tools/gpu_job.sh
export DDL_HOST_LOG=1 DDL_STAGER_LOG=1
run 120 s_p5 python bench.py --gpus 1 --steps 30 --warmup 5 --order window --idle-steps 0 --producers 5 --json-out gpurun_out/s_p5.json
run 120 s_p2 python bench.py --gpus 1 --steps 30 --warmup 5 --order window --idle-steps 0 --producers 2 --json-out gpurun_out/s_p2.json
run 120 s_sl2 python bench.py --gpus 1 --steps 30 --warmup 5 --order window --idle-steps 0 --slots 2 --json-out gpurun_out/s_sl2.json
AMD_LOG_LEVEL=3 run 120 s_log python bench.py --gpus 1 --steps 12 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/s_log.json
grep -n -i "pin\|staging\|hipMemcpyAsync\|hipHostRegister" gpurun_out/s_log.log | head -400 > gpurun_out/s_log_grep.txt || true
rm -f gpurun_out/s_log.log
