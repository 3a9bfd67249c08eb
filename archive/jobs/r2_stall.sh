source tools/gpu_job.sh
export DDL_HOST_LOG=1
run 120 s_base python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/s_base.json
run 120 s_gc python -c "import gc,sys; gc.disable(); sys.argv=['bench.py','--gpus','1','--steps','20','--warmup','5','--order','window','--idle-steps','0','--json-out','gpurun_out/s_gc.json']; import runpy; runpy.run_path('bench.py', run_name='__main__')"
run 120 s_d3 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --depth 3 --json-out gpurun_out/s_d3.json
run 120 s_w512 python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --window 512 --json-out gpurun_out/s_w512.json
run 120 s_inline python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --dispatch inline --json-out gpurun_out/s_inline.json
run 120 s_python python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --dispatch python --json-out gpurun_out/s_python.json
run 120 l_inline python bench.py --gpus 1 --order window --idle-steps 0 --dispatch inline --json-out gpurun_out/l_inline.json
run 120 l_lookahead python bench.py --gpus 1 --order window --idle-steps 0 --dispatch lookahead --json-out gpurun_out/l_lookahead.json
