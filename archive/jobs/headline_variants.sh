source tools/gpu_job.sh
run 600 kernels python -m pytest tests/test_kernels_gpu.py -q
run 200 probe python benchmarks/probe_h2d.py
run 300 bench_default python bench.py --steps 200 --warmup 20
run 300 bench_u8 python bench.py --steps 200 --warmup 20 --source-dtype uint8 --idle-steps 0
run 300 bench_w2048_p4 python bench.py --steps 200 --warmup 20 --window 2048 --producers 4 --idle-steps 0
run 300 bench_thread python -c "import os; os.environ['DDL_PRODUCER_MODE']='thread'; import sys; sys.argv=['bench.py','--steps','100','--warmup','10','--idle-steps','0']; import runpy; runpy.run_path('bench.py', run_name='__main__')"
export DDL_PRODUCER_MODE=thread
run 400 rocprof rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30
