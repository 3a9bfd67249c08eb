# Round 4, fourteenth box: the native augment/HWC dispatch tests (kind 4 fix), then: is the idle below the crossover the command processor reading host memory over a
# saturated link? A/B at fixed step times: AQL queues in device memory (HSA_ALLOCATE_QUEUE_DEV_MEM=1) and
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1), two runs each, interleaved.
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 dispatch_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "native_dispatch or augment"
SW="python benchmarks/bench_idle_sweep.py --step-ms 1.45,1.6 --floor --steps 300 --feed-steps 200"
for rep in 1 2; do
  run 200 base_$rep $SW --json-out gpurun_out/base_$rep.jsonl
  run 200 qdev_$rep env HSA_ALLOCATE_QUEUE_DEV_MEM=1 $SW --json-out gpurun_out/qdev_$rep.jsonl
  run 200 karg_$rep env HIP_FORCE_DEV_KERNARG=1 $SW --json-out gpurun_out/karg_$rep.jsonl
  run 200 both_$rep env HSA_ALLOCATE_QUEUE_DEV_MEM=1 HIP_FORCE_DEV_KERNARG=1 $SW --json-out gpurun_out/both_$rep.jsonl
done
