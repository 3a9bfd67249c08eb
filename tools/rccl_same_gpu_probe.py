"""Probe: can two RCCL ranks share one GPU on this box? (torchrun --nproc-per-node 2)

If they can, the N>1 bench path (RCCL exchange all-to-all + DDP all-reduce)
can be rehearsed on the single-GPU gpurun box before the driver's 8-GPU run.
Prints one line per rank; exits non-zero on any failure.
"""

import os
from datetime import timedelta

import torch
import torch.distributed as dist


def main() -> None:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, timeout=timedelta(seconds=60), device_id=dev)
    x = torch.arange(world * 4, dtype=torch.float32, device=dev) + 100 * rank
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    z = torch.ones(8, device=dev) * (rank + 1)
    dist.all_reduce(z)
    torch.cuda.synchronize()
    expect = torch.cat([torch.arange(rank * 4, rank * 4 + 4, dtype=torch.float32) + 100 * r for r in range(world)])
    ok = torch.equal(y.cpu(), expect) and float(z[0]) == world * (world + 1) / 2
    print(f"rank {rank}: all_to_all + all_reduce on shared cuda:0 ok={ok}", flush=True)
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
