#!/usr/bin/env python3
"""An existing map-style ``torch.utils.data.Dataset`` through ddl_amd (drop-in path).

    python examples/torch_dataset.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/torch_dataset.py

``ddl_amd.DataLoader`` is the torch-DataLoader-shaped front end of the pieces below.
``MapDatasetSource`` packs each sample (a tensor, or a flat tuple / dict of tensors, arrays and
numbers) into a byte row. ``IndexedProducer`` workers call ``dataset[i]`` for their share of every
global batch, in the world-size-invariant ``EpochOrder``. The loader hands back batches shaped like
``default_collate`` would make them, as typed views of one buffer staged on the GPU. ``state_dict()``
is the indexed cursor: resume at any world size with the same global batch.
"""

import argparse

import torch

import ddl_amd


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
    ap.add_argument("--batch-size", type=int, default=32, help="per rank")
    ap.add_argument("--epochs", type=int, default=2)
    a = ap.parse_args()

    # ddl_amd.DataLoader = start() + IndexedProducer(MapDatasetSource(dataset)) + DistributedDataLoader
    # (mode="indexed", auto_mark=True); built before the first CUDA call of the process
    with ddl_amd.DataLoader(Squares(a.n_samples), batch_size=a.batch_size, shuffle=True, num_workers=2) as dl:
        rank = dl.env.rank
        for epoch in range(a.epochs):
            seen = 0
            for img, label, weight in dl:
                assert torch.equal(img[:, 0, 0, 0].long(), label % 256)  # the sample structure survives
                seen += label.numel()
            if rank == 0:
                print(f"epoch {epoch}: {seen} samples on rank 0 as (image {tuple(img.shape)} {img.dtype}, "
                      f"label {label.dtype}, weight {weight.dtype}) on {img.device}", flush=True)


if __name__ == "__main__":
    main()
