source tools/gpu_job.sh
run 600 gpu_tests python -m pytest tests -m gpu -q
run 300 bench python bench.py
run 120 fileio python benchmarks/bench_fileio.py --n 16384 --threads 4 8 16
run 60 topo bash -c 'lspci -tv > gpurun_out/lspci_tree.txt 2>&1; for f in /sys/class/kfd/kfd/topology/nodes/*/io_links/*/properties; do echo "== $f"; cat $f; done > gpurun_out/kfd_links.txt 2>&1; nproc; free -g; df -h /dev/shm'
