# Round 4, thirteenth box: augment (RandomResizedCrop) in the native engine, vs the Python path (test oracle).
source tools/gpu_job.sh
unset DDL_BACKEND
run 400 dispatch_tests python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_loader_gpu.py -k "native_dispatch or augment"
