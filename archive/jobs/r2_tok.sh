source tools/gpu_job.sh
run 200 t_p4s1 python benchmarks/bench_tokens.py --mode pack --idle-steps 0
run 200 t_p4s2 python benchmarks/bench_tokens.py --mode pack --idle-steps 0 --slots 2
run 200 t_p8s1 python benchmarks/bench_tokens.py --mode pack --idle-steps 0 --producers 8
run 200 t_p8s2 python benchmarks/bench_tokens.py --mode pack --idle-steps 0 --producers 8 --slots 2
run 200 t_pad_p8s2 python benchmarks/bench_tokens.py --mode pad --idle-steps 0 --producers 8 --slots 2
run 200 t_python_p8s2 python benchmarks/bench_tokens.py --mode pack --idle-steps 0 --producers 8 --slots 2 --dispatch python
run 300 host_cost python tools/loader_host_cost.py
