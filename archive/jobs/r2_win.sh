source tools/gpu_job.sh
for w in 256 512 1024; do
run 120 win_$w python bench.py --gpus 1 --steps 20 --warmup 5 --window $w --order window --json-out gpurun_out/win_$w.json
run 120 winL_$w python bench.py --gpus 1 --window $w --order window --idle-steps 0 --json-out gpurun_out/winL_$w.json
done
run 120 win_256_p2 python bench.py --gpus 1 --steps 20 --warmup 5 --window 256 --producers 2 --order window --idle-steps 0 --json-out gpurun_out/win_256_p2.json
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof_final
run 300 prof_final rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30 --order window
