"""RandomResizedCrop kernel probe (for rocprofv3 PMC runs): 256 x u8 3x256x320 -> bf16 224x224."""
import torch

from ddl_amd import ops
from ddl_amd.permutation import FeistelPermutation

dev = torch.device("cuda", 0)
raw = torch.randint(0, 255, (1024, 3, 256, 320), dtype=torch.uint8, device=dev)
p = FeistelPermutation(1024, 1, 3)
for _ in range(20):
    ops.random_resized_crop(raw, perm=p, base=0, n_rows=256, size=(224, 224), seed=1, mean=[0.5] * 3, std=[0.25] * 3)
torch.cuda.synchronize()
