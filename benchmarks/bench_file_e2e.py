#!/usr/bin/env python3
"""End-to-end file-backed image feed: uint8 file -> producers -> pinned slots -> H2D -> normalised bf16.

The production path for a dataset on disk. A synthetic [N, 3, 224, 224] uint8
file is written once (then read from the page cache, or with ``--direct`` by
O_DIRECT). ``IndexedProducer`` workers gather each local batch of the
world-size-invariant global order with the native coalesced ``pread``
(``FileRowsSource``) into their pinned slots. The native stager DMAs every
slot to HBM, and the loader normalises uint8 -> bf16 on the device.

Phase 1 reports samples/s fed, with a checksum consumer that reads every
delivered byte. Phase 2 reports GPU idle % behind the PatchMLP train step.
Writes one JSON line. torchrun-compatible (each rank feeds its own GPU from
the shared file).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "ddl_amd_e2e_rows.bin"))
    ap.add_argument("--n", type=int, default=16384, help="samples in the file (16384 x 150 KB = 2.5 GB)")
    ap.add_argument("--batch", type=int, default=256, help="per-rank batch")
    ap.add_argument("--producers", type=int, default=3)
    ap.add_argument("--slots", type=int, default=2)
    ap.add_argument("--host-threads", type=int, default=4)
    ap.add_argument("--direct", action="store_true", help="O_DIRECT reads (bypass the page cache)")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--idle-steps", type=int, default=150)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd import ops
    from ddl_amd.models import FileRowsSource, IndexedProducer

    shape = (3, 224, 224)
    row = int(np.prod(shape))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if local_rank == 0 and (not os.path.exists(a.path) or os.path.getsize(a.path) != a.n * row):
        rng = np.random.default_rng(0)
        block = rng.integers(0, 255, size=(256, row), dtype=np.uint8)
        with open(a.path + ".tmp", "wb") as f:
            for c in range(0, a.n, 256):
                blk = block[: min(256, a.n - c)].copy()
                blk[:, :8] = np.arange(c, c + len(blk), dtype=np.int64).view(np.uint8).reshape(len(blk), 8)
                f.write(blk.tobytes())
        os.replace(a.path + ".tmp", a.path)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    gb = a.batch * world
    src = None
    try:
        with ddl_amd.start(n_producers=a.producers) as (env, conn):
            if env.world_size > 1:
                dist.barrier(group=env.control_group)  # the file exists before any producer opens it
            src = FileRowsSource(a.path, shape, "uint8", n=a.n, direct=a.direct)
            total = a.warmup + a.steps + a.warmup // 2 + a.idle_steps
            bpe = a.n // gb
            n_epochs = total // bpe + 2
            norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225]}
            dev = torch.device(env.device)
            dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, gb, seed=1, host_threads=a.host_threads), a.batch,
                                               conn, n_epochs, env=env, device=dev, auto_mark=True,
                                               output=ddl_amd.OutputSpec(dtype=torch.bfloat16, normalize=norm),
                                               staging=ddl_amd.StagingSpec(n_slots=a.slots),
                                               order=ddl_amd.OrderSpec(mode="indexed"))
            acc = ops.ChecksumAccumulator(dev)

            def gen():
                while True:
                    yield from dl

            it = gen()

            def barrier():
                if env.world_size > 1:
                    dist.barrier(group=env.control_group)
                torch.cuda.synchronize(dev)

            for _ in range(a.warmup):
                (x,) = next(it)
                acc.add(x)
            barrier()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                (x,) = next(it)
                acc.add(x)
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            if env.world_size > 1:
                t = torch.tensor([el], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
                el = float(t.item())
            idle = None
            if a.idle_steps:
                from ddl_amd.models.trainstep import TrainStep
                from ddl_amd.utils.tracing import ComputeIdleMeter

                step = TrainStep(dev, process_group=env.process_group if env.world_size > 1 else None)
                for _ in range(a.warmup // 2):
                    step(next(it)[0])
                meter = ComputeIdleMeter()
                barrier()
                for _ in range(a.idle_steps):
                    (x,) = next(it)
                    meter.step_begin()
                    step(x)
                    meter.step_end()
                idle = meter.result()
            st = dl.stats()
            dl.close()
            if env.rank == 0:
                print(json.dumps({
                    "bench": "file-backed e2e: uint8 file -> IndexedProducer pread -> H2D -> normalised bf16",
                    "n_gpus": env.world_size, "samples_per_s": round(a.batch * a.steps * env.world_size / el, 1),
                    "GBps_h2d": round(a.batch * a.steps * row / el / 1e9, 2), "ms_per_step": round(1e3 * el / a.steps, 4),
                    "page_cache": not a.direct, "producers": a.producers, "slots": a.slots,
                    "host_threads": a.host_threads, "file_GB": round(a.n * row / 1e9, 2),
                    "gpu_idle_pct": None if idle is None else round(idle["gpu_idle_pct"], 3),
                    "consumer_wait_s": round(st["consumer_wait_s"], 4)}), flush=True)
    finally:
        if src is not None:
            src.close()
        if local_rank == 0 and not a.keep and os.path.exists(a.path):
            os.remove(a.path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
