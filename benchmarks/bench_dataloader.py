#!/usr/bin/env python3
"""Drop-in comparison: ``ddl_amd.DataLoader`` vs ``torch.utils.data.DataLoader`` on one map-style Dataset.

Both loaders get the same ``Dataset`` object: ImageNet-shape uint8 images [3, 224, 224] with an int64
label. ``__getitem__`` returns a view of a small pre-built image table, so the dataset costs almost
nothing, and the numbers measure the loaders. The consumer is the same for both: the batch lands on the
GPU, is made contiguous there if it is a strided view, and a checksum kernel reads every image byte. The timed region is K batches after W warmup
batches, closed by a device synchronize. Then (``--idle-steps``)
the GPU idle % behind bench.py's PatchMLP train step fed by the same loader.

* ``torch``: ``DataLoader(num_workers=P, pin_memory=True, persistent_workers=True, shuffle=True)``,
  then ``.to(device, non_blocking=True)``. Workers use the spawn start method; collate runs in the
  workers and pinning in the main process's pin thread, the standard recipe.
* ``ddl``: ``ddl_amd.DataLoader(num_workers=P, shuffle=True)``. Producer processes call
  ``dataset[i]`` straight into pinned windows; the native stager copies them to HBM; batches come back
  as device views in the sample's structure.

Each implementation runs in its own process (``--impl``), so the two never share workers or the GPU
context. One JSON line per run.

    python benchmarks/bench_dataloader.py --impl ddl --workers 3
    python benchmarks/bench_dataloader.py --impl torch --workers 3
"""

from __future__ import annotations

import argparse
import json
import sys
import time

import numpy as np
import torch


class SyntheticImages(torch.utils.data.Dataset):
    """n samples of (uint8 [3, 224, 224], int64 label) over a table of `distinct` pre-built images."""

    def __init__(self, n: int, distinct: int = 64, shape=(3, 224, 224), seed: int = 0):
        self.n = int(n)
        rng = np.random.default_rng(seed)
        self.table = rng.integers(0, 256, size=(distinct, *shape), dtype=np.uint8)

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int):
        return torch.from_numpy(self.table[i % len(self.table)]), torch.tensor(i, dtype=torch.int64)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--impl", choices=["ddl", "torch"], required=True)
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--n-samples", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--host-threads", type=int, default=2,
                    help="ddl: copy threads per producer for the packed-row span copies")
    ap.add_argument("--idle-steps", type=int, default=100,
                    help="then GPU idle %% behind the bench.py PatchMLP bf16 train step fed by this loader (0: skip)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)

    ds = SyntheticImages(a.n_samples)
    if a.impl == "ddl":
        import ddl_amd

        loader = ddl_amd.DataLoader(ds, batch_size=a.batch, shuffle=True, num_workers=a.workers, seed=0,
                                    host_threads=a.host_threads)
        dev = torch.device(loader.env.device)
    else:
        loader = torch.utils.data.DataLoader(ds, batch_size=a.batch, shuffle=True, num_workers=a.workers,
                                             pin_memory=True, drop_last=True, persistent_workers=True,
                                             multiprocessing_context="spawn", prefetch_factor=4)
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")

    from ddl_amd import ops

    acc = ops.ChecksumAccumulator(dev)

    def batches():
        while True:
            for img, label in loader:
                if a.impl == "torch":
                    img = img.to(dev, non_blocking=True)
                    label = label.to(dev, non_blocking=True)
                # ddl_amd's batch views are strided over the packed (image | label) records: the
                # consumer makes the image contiguous on the device, as a model's first op would
                yield (img if img.is_contiguous() else img.contiguous()), label

    it = batches()
    for _ in range(a.warmup):
        img, _ = next(it)
        acc.add(img)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        img, label = next(it)
        acc.add(img)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    assert img.shape == (a.batch, 3, 224, 224) and img.dtype == torch.uint8 and img.device == dev
    assert label.shape == (a.batch,) and label.device == dev
    out = {"metric": "samples/s, map-style Dataset -> device batches (uint8 3x224x224 + label)",
           "impl": "ddl_amd.DataLoader" if a.impl == "ddl" else "torch.utils.data.DataLoader(pin_memory=True)",
           "workers": a.workers, "host_threads": a.host_threads if a.impl == "ddl" else None, "batch": a.batch, "steps": a.steps, "warmup": a.warmup,
           "samples_per_s": round(a.batch * a.steps / dt, 1), "ms_per_batch": round(1000 * dt / a.steps, 3),
           "h2d_gbps": round(a.batch * a.steps * 3 * 224 * 224 / dt / 1e9, 2), "device": str(dev)}
    if a.idle_steps and dev.type == "cuda":
        from ddl_amd.models.trainstep import TrainStep
        from ddl_amd.utils.tracing import ComputeIdleMeter

        step = TrainStep(dev, dim=384, depth=4)

        def prep(x):  # uint8 -> bf16 in [0, 1] on the device (the model's input)
            return x.to(torch.bfloat16).mul_(1.0 / 255)

        for _ in range(5):
            step(prep(next(it)[0]))
        meter = ComputeIdleMeter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        for _ in range(a.idle_steps):
            img, _ = next(it)
            meter.step_begin()
            step(prep(img))
            meter.step_end()
        torch.cuda.synchronize(dev)
        res = meter.result()
        out["gpu_idle_pct"] = round(res["gpu_idle_pct"], 2)
        out["train_step"] = {"model": "PatchMLP dim=384 depth=4 fwd+bwd+SGD bf16 (bench.py phase 2)",
                             "samples_per_s": round(a.batch * a.idle_steps / (time.perf_counter() - t2), 1)}
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "a") as f:
            f.write(line + "\n")
    if a.impl == "ddl":
        loader.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
