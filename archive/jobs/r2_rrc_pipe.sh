# RandomResizedCrop: software-pipelined persistent workgroups (band i+1 staged while band i resamples).
source tools/gpu_job.sh
run 300 rrc_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_loader_gpu.py -k "random_resized_crop or augment" -m gpu
for n in 2 3 4 6; do
  export DDL_RRC_WG_PER_CU=$n; run 120 kernels_wg$n python benchmarks/kernels_bench.py
done
unset DDL_RRC_WG_PER_CU
run 240 resident_aug python benchmarks/bench_resident.py --dtype uint8 --augment
