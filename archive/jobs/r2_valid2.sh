source tools/gpu_job.sh
run 900 gpu_all python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_driver python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/bench_driver.json
run 300 bench_default python bench.py --json-out gpurun_out/bench_default.json
rm -rf gpurun_out/prof_final
run 300 prof_final rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30 --order window
