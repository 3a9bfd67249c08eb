#!/usr/bin/env python3
"""An existing map-style ``torch.utils.data.Dataset`` through ddl_amd (drop-in path).

    python examples/torch_dataset.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/torch_dataset.py

``MapDatasetSource`` packs each sample (a tensor, or a flat tuple / dict of tensors, arrays and
numbers) into a byte row. ``IndexedProducer`` workers call ``dataset[i]`` for their share of every
global batch, in the world-size-invariant ``EpochOrder``. The loader hands back batches shaped like
``default_collate`` would make them, as typed views of one buffer staged on the GPU. ``state_dict()``
is the indexed cursor: resume at any world size with the same global batch.
"""

import argparse

import torch

import ddl_amd
from ddl_amd.models import IndexedProducer, MapDatasetSource


class Squares(torch.utils.data.Dataset):
    """A stand-in for user code: (image uint8 [3, 32, 32], label int, weight float)."""

    def __init__(self, n: int):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        img = torch.full((3, 32, 32), i % 256, dtype=torch.uint8)
        return img, i, 1.0 / (1 + i)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-samples", type=int, default=2048)
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=2)
    a = ap.parse_args()

    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(MapDatasetSource(Squares(a.n_samples)), a.global_batch),
                                           a.global_batch // env.world_size, conn, a.epochs, mode="indexed", env=env,
                                           auto_mark=True)
        for epoch in range(a.epochs):
            seen = 0
            for img, label, weight in dl:
                assert torch.equal(img[:, 0, 0, 0].long(), label % 256)  # the sample structure survives
                seen += label.numel()
            if env.rank == 0:
                print(f"epoch {epoch}: {seen} samples on rank 0 as (image {tuple(img.shape)} {img.dtype}, "
                      f"label {label.dtype}, weight {weight.dtype}) on {img.device}", flush=True)


if __name__ == "__main__":
    main()
