#!/usr/bin/env python3
"""The reference's own workload (BASELINE config 1 shape) on the GPU path.

The reference harness (tests/run_ddl.py): 3 producers per GPU, each holding a
(100,520 x 9) f32 shard with column groups (3, 5, 1), batch 4096, a CPU
``rng.shuffle`` of the whole window every round. Its measured ceiling is
3.90M rows/s per GPU group (three parallel host shuffles, no H2D).

Here the same producers fill their windows once (static shard, like the
reference's ``post_init``); every round the window is re-staged H2D and the
consumer gets device-shuffled, contiguous (pos, target, weight) groups from
one fused gather+split kernel. The consumer step touches every delivered byte
(streaming checksum). Prints one JSON line with rows/s.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

REF_ROWS_PER_S = 3.90e6  # SURVEY §6, reference ceiling at P=3 (CI shape)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=480)
    ap.add_argument("--warmup", type=int, default=48)
    ap.add_argument("--producers", type=int, default=3)
    ap.add_argument("--timesteps", type=int, default=10, help="reference nData (10052 rows each)")
    ap.add_argument("--host-shuffle", action="store_true",
                    help="also run the reference's per-round CPU rng.shuffle in the producers")
    ap.add_argument("--consumer", default="flat", choices=["flat", "groups"],
                    help="flat: ONE streaming checksum over the batch's three groups (adjacent in one allocation); "
                         "groups: one checksum launch per group")
    ap.add_argument("--dispatch", default="native", choices=["native", "inline", "lookahead", "window", "python"])
    a = ap.parse_args(argv)

    import torch

    import ddl_amd
    from ddl_amd import Marker, ops
    from ddl_amd.models import PointwiseProducer

    with ddl_amd.start(n_producers=a.producers) as (env, conn):
        dev = torch.device(env.device)
        producer = PointwiseProducer(n_timesteps=a.timesteps, host_shuffle=a.host_shuffle)
        dl = ddl_amd.DistributedDataLoader(producer, 4096, conn, 10 ** 6, 0.0, "alltoall", env.rank, env.world_size,
                                           env=env, output=ddl_amd.OutputSpec(contiguous=True),
                                           staging=ddl_amd.StagingSpec(
                                               native_dispatch={"native": True, "python": False}.get(a.dispatch,
                                                                                                     a.dispatch)),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=1))
        acc = ops.ChecksumAccumulator(dev)

        def consume(groups):
            if a.consumer == "groups" or dev.type != "cuda":
                for g in groups:
                    acc.add(g)
                return
            g0 = groups[0]
            n = sum(g.numel() for g in groups)
            off = g0.storage_offset()
            assert all(g.untyped_storage().data_ptr() == g0.untyped_storage().data_ptr() for g in groups)
            assert [g.storage_offset() for g in groups] == [off, off + groups[0].numel(),
                                                             off + groups[0].numel() + groups[1].numel()]
            acc.add(g0.new_empty(0).set_(g0.untyped_storage(), off, (n,)))

        def batches():
            while True:
                for i in range(len(dl)):
                    yield dl[i]
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)

        it = batches()

        def sync():
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)

        for _ in range(a.warmup):
            consume(next(it))
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            consume(next(it))
        sync()
        dt = time.perf_counter() - t0
        rows = 4096 * a.steps * env.world_size
        mode = (dl.stats().get("native_dispatch") or {}).get("mode")
        dl.close()
        if env.rank == 0:
            print(json.dumps({"bench": "pointwise (reference CI shape)", "rows_per_s": round(rows / dt),
                              "batches_per_s": round(a.steps / dt, 1), "us_per_batch": round(1e6 * dt / a.steps, 1),
                              "vs_reference_ceiling": round(rows / dt / (REF_ROWS_PER_S * env.world_size), 2),
                              "batches_per_window": len(dl), "producers": a.producers, "host_shuffle": a.host_shuffle,
                              "consumer": a.consumer, "dispatch": a.dispatch, "mode": mode,
                              "device": str(dev)}))


if __name__ == "__main__":
    main()
