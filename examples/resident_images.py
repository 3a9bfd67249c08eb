#!/usr/bin/env python3
"""HBM-resident image dataset with an exact global shuffle (and on-device augmentation on a GPU).

    python examples/resident_images.py                       # 1 GPU (or CPU, without augmentation)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/resident_images.py

The dataset lives in node-shared memory here (``SharedArraySource``); with a
real dataset use ``FileRowsSource.from_npy(path)`` or ``FileRowsSource(path,
shape, "uint8")`` instead. The dataset goes into HBM once: an ImageNet-size uint8
set is 193 GB at 3x224x224, which fits one MI355X, so by default (``replicate="auto"``)
every rank holds a full replica -- it loads 1/W of it from the host and RCCL
all-gathers over xGMI fill in the rest -- and no step moves a row between GPUs.
(``--replicate false``, or a dataset too big for HBM: each rank holds a shard and
every step all-to-alls 7/8 of its batch over xGMI.) Every epoch the loader
delivers rank r's slice of the world-size-invariant global order. On a GPU each batch is
RandomResizedCrop + flip + normalise + cast to bf16, in one kernel. The loader
state is a checkpointable cursor: resume with ``resume_state=``, at any world
size.
"""

import argparse
import os

import numpy as np
import torch

import ddl_amd
from ddl_amd.models import SharedArraySource
from ddl_amd.models.trainstep import TrainStep
from ddl_amd.resident import ResidentGlobalLoader


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-samples", type=int, default=2048)
    ap.add_argument("--hw", type=int, default=80, help="stored image side (uint8, CHW)")
    ap.add_argument("--crop", type=int, default=64, help="crop side (a multiple of the 16-px patch)")
    ap.add_argument("--global-batch", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--replicate", default="auto", choices=["auto", "true", "false"])
    a = ap.parse_args()

    name = f"ddl_amd_example_imgs_{os.environ.get('MASTER_PORT', os.getpid())}"
    shape = (3, a.hw, a.hw)
    creator = int(os.environ.get("LOCAL_RANK", "0")) == 0
    if creator:
        rng = np.random.default_rng(0)
        data = rng.integers(0, 255, (a.n_samples, *shape), dtype=np.uint8)
        src = SharedArraySource.create(name, torch.from_numpy(data))
    with ddl_amd.start(n_producers=0) as (env, _):
        if env.world_size > 1:
            torch.distributed.barrier(group=env.control_group)
        if not creator:
            src = SharedArraySource(name, a.n_samples, shape, "uint8")
        gpu = env.device.startswith("cuda")
        norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225]}
        dl = ResidentGlobalLoader(src, a.global_batch, env, seed=0, n_epochs=a.epochs, depth=2,
                                  out_dtype=torch.bfloat16 if gpu else torch.float32, normalize=norm,
                                  augment={"size": (a.crop, a.crop)} if gpu else None,
                                  replicate={"auto": "auto", "true": True, "false": False}[a.replicate])
        step = TrainStep(env.device, dim=64, depth=1, dtype=torch.bfloat16 if gpu else torch.float32,
                         process_group=env.process_group if env.world_size > 1 else None) if gpu else None
        for epoch in range(a.epochs):
            n = 0
            for batch in dl:  # [global_batch / W, 3, crop, crop] on this rank's device
                if step is not None:
                    step(batch)
                n += batch.shape[0]
            if env.rank == 0:
                print(f"epoch {epoch}: {n} samples on rank 0, batch {tuple(batch.shape)} {batch.dtype}, "
                      f"cursor {dl.state_dict()['epoch']}/{dl.state_dict()['global_batch_cursor']}, "
                      f"{'replicated' if dl.replicated else 'sharded'}", flush=True)
        dl.close()
    src.close()  # unlinks the segment only in the process that created it


if __name__ == "__main__":
    main()
