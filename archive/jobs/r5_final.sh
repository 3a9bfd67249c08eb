# Round 5, final tree: whole GPU suite, smoke, the driver's command x2, a rocprofv3 kernel-trace summary of
# the driver's command (producers as threads under the profiler), the kernel benchmark with its hardware
# counters (one --pmc pass per counter group, kernel trace only), and the native per-batch host cost at the
# reference's CI shape.
source tools/gpu_job.sh
unset DDL_BACKEND
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 bench_a python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_a.json
run 200 bench_b python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b.json
run 120 kbench python benchmarks/kernels_bench.py
run 200 pw_window python benchmarks/bench_pointwise.py --dispatch window
run 300 host_cost env STEPS=3000 python tools/loader_host_cost.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 400 rocprof env DDL_PRODUCER_MODE=thread rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 100 --warmup 10 --json-out gpurun_out/bench_prof.json
run 300 pmc_fetch rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc1 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 300 pmc_write rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc2 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 300 pmc_insts rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc3 -o k --output-format csv -- python3 benchmarks/kernels_bench.py
run 60 pmc_summary python tools/pmc_summary.py gpurun_out/pmc_summary.json gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
