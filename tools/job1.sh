source tools/gpu_job.sh
run 400 build python -c "import __graft_entry__ as g; g.build()"
run 600 kernels python -m pytest tests/test_kernels_gpu.py -x -q
run 300 loader python -m pytest tests/test_loader_gpu.py -x -q
run 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 200 probe python benchmarks/probe_h2d.py
run 400 bench python bench.py --steps 100 --warmup 10
