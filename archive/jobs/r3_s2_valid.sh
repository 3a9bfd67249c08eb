# Round 3, session 2: validation of the tree with the auto copy policy and pro-rata accounting: full GPU suite,
# smoke, driver config, token sweep, rocprofv3 kernel / memory-copy stats of the headline.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  run 120 v_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/v_drv_$i.json
done
run 300 v_sw_tok python benchmarks/bench_idle_sweep.py --family tokens --ratios 0.5,0.75,0.9,1.1,1.5 --floor --json-out gpurun_out/v_sw_tok.jsonl
export DDL_PRODUCER_MODE=thread
rm -rf gpurun_out/prof_s2
run 400 rocprof_s2 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_s2 -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --idle-steps 30 --order window
run 120 dma_probe python benchmarks/probe_dma_gather.py
