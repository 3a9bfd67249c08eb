# Round 3, session 2: auto policy keyed on ring wait AND an idle link: slots 1 vs 2 in the driver configuration,
# and the idle sweep below the crossover.
source tools/gpu_job.sh
for i in 1 2 3 4; do
  run 120 sm1_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --slots 1 --json-out gpurun_out/sm1_$i.json
  run 120 sm2_$i python bench.py --gpus 1 --steps 20 --warmup 5 --order window --idle-steps 0 --slots 2 --json-out gpurun_out/sm2_$i.json
done
R="--ratios 0.5,0.75,0.9,1.25 --floor"
run 300 sm_sw_bf16 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/sm_sw_bf16.jsonl
run 300 sm_sw_u8 python benchmarks/bench_idle_sweep.py --source-dtype uint8 $R --json-out gpurun_out/sm_sw_u8.jsonl
run 300 sm_tok python benchmarks/bench_tokens.py --batch 2048 --steps 300 --warmup 30 --idle-steps 0
run 300 sm_policy python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -m gpu -k "copy_stream_policies or interval"
