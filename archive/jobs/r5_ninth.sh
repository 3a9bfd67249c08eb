# Round 5, ninth box: loader / exchange / direct-DMA GPU tests after the engine-release change, incl. the
# stuck copy with the exchange on.
source tools/gpu_job.sh
unset DDL_BACKEND
run 700 tests python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_exchange_gpu.py tests/test_direct_dma_gpu.py tests/test_loader_gpu.py -m gpu
