# Round 3: step-boundary idle vs the hardware-queue layout of the loader's streams.
source tools/gpu_job.sh
R="--ratios 0.5,0.75 --floor"
run 200 q4 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/q4.jsonl
run 200 q8 env GPU_MAX_HW_QUEUES=8 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/q8.jsonl
run 200 q16 env GPU_MAX_HW_QUEUES=16 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/q16.jsonl
run 200 q4_nowarm env DDL_WARM_SDMA=0 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/q4_nowarm.jsonl
run 200 q4_cs1 env DDL_COPY_STREAMS=1 python benchmarks/bench_idle_sweep.py $R --json-out gpurun_out/q4_cs1.jsonl
run 200 q8_probe env GPU_MAX_HW_QUEUES=8 python benchmarks/probe_handoff.py --variants held,h2d_gather,h2d_gather_devwait
