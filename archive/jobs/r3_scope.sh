# Round 3: the residual below the crossover is the compute stream's per-step cross-stream wait
# (~28 us more per step boundary than the meter's own floor, trace_floor). A/B the scope of the
# engine's event release.
source tools/gpu_job.sh
run 200 t_inline2 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "two_streams or other_streams" -m gpu
for sc in system device nofence; do
  run 300 sc_$sc env DDL_EVENT_SCOPE=$sc python benchmarks/bench_idle_sweep.py --floor --ratios 0.5,0.75,0.9,1.25 --json-out gpurun_out/sc_$sc.jsonl
done
for sc in system device nofence; do
  run 200 bd_$sc env DDL_EVENT_SCOPE=$sc python bench.py --gpus 1 --steps 20 --warmup 5 --order window --json-out gpurun_out/bd_$sc.json
done
