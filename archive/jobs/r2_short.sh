# Timeline of the driver's short headline run (20 steps): copies, kernels and roctx phases.
source tools/gpu_job.sh
export DDL_PRODUCER_MODE=thread
for w in 256 1024; do
rm -rf gpurun_out/short_$w
run 300 short_$w rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/short_$w -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --window $w --idle-steps 0 --order window --json-out gpurun_out/short_$w.json
done
unset DDL_PRODUCER_MODE
for i in 1 2 3; do run 120 drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/drv_$i.json; done
run 120 drv_w1024 python bench.py --gpus 1 --steps 20 --warmup 5 --window 1024 --json-out gpurun_out/drv_w1024.json
