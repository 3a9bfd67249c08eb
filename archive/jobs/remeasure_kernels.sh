# Host facts + re-measure the loader kernels, token pad/pack and RRC after the latest kernel changes.
source tools/gpu_job.sh
{ df -h /dev/shm; free -g; nproc; cat /proc/sys/kernel/yama/ptrace_scope 2>/dev/null; ulimit -l; } > gpurun_out/host_facts.txt 2>&1
run 300 kernels python benchmarks/kernels_bench.py
run 300 tok_pack python benchmarks/bench_tokens.py --mode pack --steps 1000 --warmup 50
run 300 tok_pad python benchmarks/bench_tokens.py --mode pad --steps 1000 --warmup 50
