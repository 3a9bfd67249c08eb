#!/usr/bin/env python3
"""Per-batch HOST cost of the loader's consumer path (GPU box): native dispatch vs the Python path.

Runs the reference CI shape (pointwise: 3 producers x 100,520 x 9 f32 windows, batch 4096, device
shuffle, contiguous (3, 5, 1) groups) and the image headline shape (3x224x224 bf16, batch 256), with
``dl[i]`` + ``mark`` and NO consumer kernel, and reports per batch:

* ``thread_cpu_us``: CPU time of the consumer thread (``time.thread_time``) -- what the Python /
  native dispatch costs the host, excluding time asleep in futex / condition-variable waits;
* ``wall_us``: wall time (bounded below by the batch kernel on the GPU and by the feed).

One JSON line per (shape, dispatch).
"""

from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(shape: str, native, steps: int) -> dict:
    import torch

    import ddl_amd
    from ddl_amd.specs import from_flat
    from ddl_amd import Marker
    from ddl_amd.models import PointwiseProducer
    from ddl_amd.models.producers import ImageWindowProducer

    if shape == "tokens":
        return run_tokens(native, steps)
    with ddl_amd.start(n_producers=3) as (env, conn):
        dev = torch.device(env.device)
        if shape == "pointwise":
            prod, bs, kw = PointwiseProducer(n_timesteps=10, host_shuffle=False), 4096, dict(contiguous=True)
        else:
            prod, bs, kw = ImageWindowProducer(256, (3, 224, 224), "bfloat16", refill="stamp"), 256, \
                dict(out_dtype=torch.bfloat16)
        dl = ddl_amd.DistributedDataLoader(prod, bs, conn, 10 ** 6, env=env, device=dev,
                                           **from_flat(dict(kw, native_dispatch=native, shuffle="device", seed=1)))

        def batches():
            while True:
                for i in range(len(dl)):
                    yield dl[i]
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)

        it = batches()
        for _ in range(200):
            next(it)
        torch.cuda.synchronize()
        c0, w0 = time.thread_time(), time.perf_counter()
        for _ in range(steps):
            next(it)
        c1, w1 = time.thread_time(), time.perf_counter()
        st = dl.stats()
        torch.cuda.synchronize()
        dl.close()
    return {"shape": shape, "dispatch": native if native else "python", "batches": steps,
            "thread_cpu_us": round(1e6 * (c1 - c0) / steps, 2), "wall_us": round(1e6 * (w1 - w0) / steps, 2),
            "engine": st.get("native_dispatch")}


def run_tokens(native, steps: int, producers: int = 4, k: int = 8) -> dict:
    """Config 4 shape: 64 sequences (seq_len 4096, mean ~2.2k tokens) per batch, packed, k batches per window."""
    import torch

    import ddl_amd
    from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer

    src = SharedTokenSource.synthetic(f"ddl_amd_lhc_{os.getpid()}", 8192, 256, 4096, seed=1)
    try:
        with ddl_amd.start(n_producers=producers) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(
                TokenBatchProducer(src, 64, 4096, "pack", pack_order="ffd", batches_per_window=k), 64, conn, 10 ** 4,
                env=env, auto_mark=True, output=ddl_amd.OutputSpec(collate="tokens"),
                staging=ddl_amd.StagingSpec(native_dispatch=native), order=ddl_amd.OrderSpec(mode="indexed"))

            def gen():
                while True:
                    yield from dl

            it = gen()
            for _ in range(200):
                next(it)
            torch.cuda.synchronize()
            c0, w0 = time.thread_time(), time.perf_counter()
            for _ in range(steps):
                next(it)
            c1, w1 = time.thread_time(), time.perf_counter()
            st = dl.stats()
            torch.cuda.synchronize()
            dl.close()
    finally:
        src.close()
    return {"shape": f"tokens (64 seqs packed, {producers} producers, {k} batches per window)", "dispatch": native if native else "python",
            "batches": steps, "thread_cpu_us": round(1e6 * (c1 - c0) / steps, 2),
            "wall_us": round(1e6 * (w1 - w0) / steps, 2), "consumer_wait_s": round(st["consumer_wait_s"], 4),
            "engine": st.get("native_dispatch")}


def main() -> int:
    steps = int(os.environ.get("STEPS", "3000"))
    for shape in ("pointwise", "images", "tokens"):
        for native in ("window", "inline", "lookahead", False):
            print(json.dumps(run(shape, native, steps // 5 if shape == "images" else steps)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
