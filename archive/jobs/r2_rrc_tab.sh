# RandomResizedCrop fast path with per-band LDS x tables: correctness, kernel time, resident augment.
source tools/gpu_job.sh
run 300 rrc_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_loader_gpu.py -k "random_resized_crop or augment" -m gpu
run 180 kernels python benchmarks/kernels_bench.py
run 120 rrc_prof rocprofv3 --kernel-trace --stats -d gpurun_out/rrc_prof -o rrc -- python3 tools/rrc_probe.py
run 240 resident_aug python benchmarks/bench_resident.py --dtype uint8 --augment
