# The usage examples on the GPU (augmentation + train step on the resident path; device pad/pack for tokens).
source tools/gpu_job.sh
run 200 ex_resident python examples/resident_images.py
run 200 ex_tokens_pack python examples/tokens_packed.py
run 200 ex_tokens_pad python examples/tokens_packed.py --mode pad
