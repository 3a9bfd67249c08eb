source tools/gpu_job.sh
for i in 1 2; do
run 120 cs1_$i env DDL_COPY_STREAMS=1 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/cs1_$i.json
run 120 cs2_$i env DDL_COPY_STREAMS=2 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/cs2_$i.json
done
run 120 cs1_long env DDL_COPY_STREAMS=1 python bench.py --gpus 1 --order window --idle-steps 0 --json-out gpurun_out/cs1_long.json
run 120 cs2_long env DDL_COPY_STREAMS=2 python bench.py --gpus 1 --order window --idle-steps 0 --json-out gpurun_out/cs2_long.json
run 400 cs2_tests env DDL_COPY_STREAMS=2 python -u -m pytest tests/test_loader_gpu.py tests/test_checkpoint.py -x -q --timeout 120 --timeout-method thread -m gpu
export DDL_COPY_STREAMS=2
rm -rf gpurun_out/prof_cs2
run 300 prof_cs2 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_cs2 -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 0 --order window
