#!/bin/bash
# Round 6: where the pressure-phase idle of the window path sits (per-step device gaps vs host timings):
# hardware queues per process (GPU_MAX_HW_QUEUES, default 4) and the stream -> queue map (spare streams).
source tools/gpu_job.sh
run 120 q4_a python tools/pressure_gaps.py --copy-timing
run 120 q4_s1 python tools/pressure_gaps.py --copy-timing --spare-streams 1
run 120 q4_s2 python tools/pressure_gaps.py --copy-timing --spare-streams 2
run 120 q4_s3 python tools/pressure_gaps.py --copy-timing --spare-streams 3
run 120 q8 env GPU_MAX_HW_QUEUES=8 python tools/pressure_gaps.py --copy-timing
run 120 q16 env GPU_MAX_HW_QUEUES=16 python tools/pressure_gaps.py --copy-timing
run 120 q4_b python tools/pressure_gaps.py --copy-timing
