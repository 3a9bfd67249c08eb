# Round 5, thirty-first box: every usage example on the GPU (the CPU suite runs them over gloo on the CPU).
source tools/gpu_job.sh
unset DDL_BACKEND
run 200 ex_run_ddl python examples/run_ddl.py
run 200 ex_resident python examples/resident_images.py --n-samples 2048 --epochs 2
run 200 ex_tokens python examples/tokens_packed.py --n-seqs 1024 --epochs 2
run 200 ex_torch_dataset python examples/torch_dataset.py --epochs 3
