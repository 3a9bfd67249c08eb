#!/bin/bash
# Round 6: output block size of the batch engine and the indexed loaders (one allocator event on the compute
# stream per freed block): 512 MB (default, 6 batches of 77 MB) vs 2 GB (26) vs 8 GB (106), window and zero-copy.
source tools/gpu_job.sh
for i in 1 2; do
  for mb in 512 2048 8192; do
    run 120 win_${mb}_$i python tools/pressure_gaps.py --meter plain --copy-timing --block-mb $mb
    run 120 zc_${mb}_$i python tools/pressure_gaps.py --path zero_copy --meter plain --block-mb $mb
  done
done
