# Round 3, session 2: final validation of the session's tree (GPU suite, smoke, driver config 3x), plus the
# indexed-phase probe.
source tools/gpu_job.sh
run 900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  run 120 f_drv_$i python bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/f_drv_$i.json
done

