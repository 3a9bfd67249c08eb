# Round 3: step-boundary idle, the loader's hand-off pattern rebuilt without the loader.
source tools/gpu_job.sh
run 200 ph2 python benchmarks/probe_handoff.py --variants held,side_gather,h2d_gather,h2d_gather_nowait,h2d_gather_devwait
