# Round 5, tenth box: the reference's two-partner exchange (sendrecv_replace: grouped isend / irecv) through
# a 1-rank RCCL group, in the loader tests and in the driver's bench; the all-to-all for comparison.
source tools/gpu_job.sh
unset DDL_BACKEND
run 300 tests python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_exchange_gpu.py -m gpu -k "exchange_enabled"
run 200 exch_srr env DDL_BACKEND=nccl python bench.py --steps 100 --warmup 10 --exchange 0.5 --exchange-method sendrecv_replace --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/exch_srr.json
run 200 exch_a2a env DDL_BACKEND=nccl python bench.py --steps 100 --warmup 10 --exchange 0.5 --idle-steps 0 --order window --pressure-ratio 0 --json-out gpurun_out/exch_a2a.json
