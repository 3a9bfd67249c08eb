#!/usr/bin/env python3
"""An existing map-style ``torch.utils.data.Dataset`` through ddl_amd: a DDP training loop with a training
and an evaluation loader (the drop-in path).

    python examples/torch_dataset.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/torch_dataset.py

``ddl_amd.DataLoader`` takes torch's ``DataLoader`` arguments. Underneath, ``MapDatasetSource`` packs each
sample (a tensor, or a flat tuple / dict of tensors, arrays and numbers) into a byte row; ``IndexedProducer``
workers call ``dataset[i]`` for their share of every global batch, in the world-size-invariant ``EpochOrder``;
the loader hands back batches shaped like ``default_collate`` would make them, as typed views of one buffer
staged on the GPU. ``batch_size`` is per rank (as with ``DistributedSampler``). Both loaders belong to one
launcher session: the process group the first one creates carries the DDP model, and it stays up until the
last loader closes. ``state_dict()`` is the indexed cursor: resume at any world size with the same global
batch.
"""

import argparse

import torch
import torch.distributed as dist

import ddl_amd


class Squares(torch.utils.data.Dataset):
    """A stand-in for user code: (image uint8 [3, 32, 32], label int, weight float); the class to learn is the
    image's brightness bin, (label % 256) // 26."""

    def __init__(self, n: int, offset: int = 0):
        self.n, self.offset = n, offset

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        j = i + self.offset
        img = torch.full((3, 32, 32), j % 256, dtype=torch.uint8)
        return img, j, 1.0 / (1 + j)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-samples", type=int, default=2048)
    ap.add_argument("--batch-size", type=int, default=32, help="per rank")
    ap.add_argument("--epochs", type=int, default=2)
    a = ap.parse_args()

    # torch's arguments; the training loader shuffles, the evaluation loader keeps the dataset order
    train = ddl_amd.DataLoader(Squares(a.n_samples), batch_size=a.batch_size, shuffle=True, num_workers=2,
                               pin_memory=True, persistent_workers=True, seed=0)
    val = ddl_amd.DataLoader(Squares(a.n_samples // 4, offset=a.n_samples), batch_size=a.batch_size,
                             num_workers=1)
    env, dev = train.env, torch.device(train.env.device)
    model = torch.nn.Sequential(torch.nn.Linear(1, 64), torch.nn.ReLU(), torch.nn.Linear(64, 10)).to(dev)
    if env.world_size > 1:  # the session's DP group (RCCL on GPUs, gloo on CPUs)
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if dev.type == "cuda"
                                                          else None)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)

    def features(img):  # the image's value in [0, 1]: one pixel is enough for this toy task
        return img[:, 0, 0, :1].float() / 255

    for epoch in range(a.epochs):
        model.train()
        seen = 0
        for img, label, weight in train:
            assert torch.equal(img[:, 0, 0, 0].long(), label % 256)  # the sample structure survives
            loss = torch.nn.functional.cross_entropy(model(features(img)), (label % 256) // 26)
            opt.zero_grad()
            loss.backward()
            opt.step()
            seen += label.numel()
        model.eval()
        stats = torch.zeros(2, device=dev)  # summed eval loss, samples
        with torch.no_grad():
            for img, label, _ in val:
                klass = (label % 256) // 26
                stats[0] += torch.nn.functional.cross_entropy(model(features(img)), klass, reduction="sum")
                stats[1] += label.numel()
        if env.world_size > 1:
            dist.all_reduce(stats, group=env.process_group)
        if env.rank == 0:
            print(f"epoch {epoch}: {seen} samples on rank 0 as (image {tuple(img.shape)} {img.dtype}, "
                  f"label {label.dtype}, weight {weight.dtype}) on {img.device}; eval loss "
                  f"{float(stats[0] / stats[1]):.3f} over {int(stats[1])} samples", flush=True)
    ckpt = train.state_dict()  # resumable: ddl_amd.DataLoader(..., resume_state=ckpt), at any world size
    train.close()
    val.close()  # the session (process groups, job watchdog) ends with the last loader
    if env.rank == 0:
        print(f"checkpoint cursor: epoch {ckpt['epoch']}, global batch {ckpt['global_batch_cursor']}",
              flush=True)


if __name__ == "__main__":
    main()
