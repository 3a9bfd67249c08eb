# Round 4, twentieth box: why direct-DMA staging was refused on the nineteenth box (reason string), then its
# correctness test and the idle A/B if it runs.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 direct_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "direct_dma" -m gpu
