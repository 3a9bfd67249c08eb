#!/usr/bin/env python3
"""BASELINE config 1: synthetic TensorDataset 1k x 3x32x32, world_size 2, CPU plumbing.

The reference runs this shape under ``mpirun`` on the CPU to check its
protocol; no throughput is published for it. Here every rank is
a torchrun process on the gloo backend (``DDL_DEVICE=cpu``) with P producer
workers. The dataset sits in node-shared memory (``SharedArraySource``), and
the indexed producers deliver the world-size-invariant global order.

Per epoch the bench checks exactly-once delivery: the union of all ranks'
sample ids is every id once, gathered over the gloo control group. It then
reports samples/s over all ranks.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        benchmarks/bench_plumbing.py
"""

import argparse
import json
import os
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-samples", type=int, default=1000)
    ap.add_argument("--global-batch", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--producers", type=int, default=2)
    a = ap.parse_args(argv)
    os.environ.setdefault("DDL_DEVICE", "cpu")

    import numpy as np
    import torch
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd.models import IndexedProducer, SharedArraySource

    shape = (3, 32, 32)
    name = f"ddl_amd_benchplumb_{os.environ.get('MASTER_PORT', '0')}"
    creator = int(os.environ.get("LOCAL_RANK", "0")) == 0
    if creator:  # sample i: every value = i (float32), so a batch row names its sample
        data = torch.arange(a.n_samples, dtype=torch.float32).view(-1, 1, 1, 1).expand(-1, *shape).contiguous()
        src = SharedArraySource.create(name, data)
    try:
        with ddl_amd.start(n_producers=a.producers) as (env, conn):
            if env.world_size > 1:
                dist.barrier(group=env.control_group)  # the creator's segment exists before anyone opens it
            if not creator:
                src = SharedArraySource(name, a.n_samples, shape, "float32")
            lb = a.global_batch // env.world_size
            # one epoch more than is timed: the loader shuts its producers down at the end of its last epoch,
            # and that teardown (process exits) is not plumbing throughput
            dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, a.global_batch, seed=3), lb, conn, a.epochs + 1,
                                               env=env, auto_mark=True, order=ddl_amd.OrderSpec(mode="indexed"))
            bpe = dl.windows_per_epoch
            exact = True
            t0 = time.perf_counter()
            for _ in range(a.epochs):
                ids = torch.cat([b[:, 0, 0, 0].to(torch.int64) for (b,) in dl])
                if env.world_size > 1:
                    parts = [torch.empty_like(ids) for _ in range(env.world_size)]
                    dist.all_gather(parts, ids, group=env.control_group)
                    ids = torch.cat(parts)
                got = np.sort(ids.numpy())
                exact &= bool(np.array_equal(got, np.unique(got)) and len(got) == bpe * a.global_batch)
            el = time.perf_counter() - t0
            if env.world_size > 1:
                t = torch.tensor([el], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
                el = float(t.item())
            dl.close()
            if env.rank == 0:
                print(json.dumps({
                    "bench": "config 1 plumbing: 1k x 3x32x32 f32, indexed global order, CPU/gloo",
                    "world_size": env.world_size, "producers_per_rank": a.producers, "epochs": a.epochs,
                    "global_batch": a.global_batch, "samples_per_s": round(a.epochs * bpe * a.global_batch / el, 1),
                    "exactly_once_every_epoch": exact}), flush=True)
    finally:
        if creator:
            src.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
