#!/bin/bash
# Round 6: the window path's pressure gaps under the three ways of timing the steps (bench.py's meter makes
# its events per step; the diagnostic makes them up front and queries the previous step's end).
source tools/gpu_job.sh
for i in 1 2; do
  run 120 late_$i python tools/pressure_gaps.py --copy-timing --meter late
  run 120 plain_$i python tools/pressure_gaps.py --copy-timing --meter plain
  run 120 bench_$i python tools/pressure_gaps.py --copy-timing --meter bench
done
