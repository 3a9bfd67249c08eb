# Round 3, session 2: re-validate the restored tree (full GPU suite, smoke, driver config 3x), then the
# adaptive copy-stream policy vs strict alternation on the tuned idle sweep.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  run 120 s2_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/s2_drv_$i.json
done
R="--ratios 0.5,0.75,0.9,1.25 --floor"
run 300 cp_adaptive python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/cp_adaptive.jsonl
run 300 cp_alternate env DDL_COPY_POLICY=alternate python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/cp_alternate.jsonl
run 300 cp_u8_adaptive python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/cp_u8_adaptive.jsonl
run 300 cp_u8_alternate env DDL_COPY_POLICY=alternate python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/cp_u8_alternate.jsonl
