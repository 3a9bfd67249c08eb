#!/usr/bin/env python3
"""Reference-style usage of ddl_amd (the analogue of the reference's tests/run_ddl.py).

    python examples/run_ddl.py                      # 1 rank: consumer + 3 producers (mpirun -np 4 layout)
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/run_ddl.py    # 2 DP ranks

The user writes a ProducerFunctionSkeleton subclass (load a shard in on_init,
fill the window in post_init, refresh it in execute_function), decorates
``main`` with ``@distributed_dataloader`` and drives the loader with
``mark(END_OF_BATCH / END_OF_EPOCH)``. Unlike the reference, batches arrive on
the GPU (staged over the prefetch stream) when one is present, the producer
shuffle happens on the device (``shuffle="device"``), and the global shuffle
exchange actually runs across ranks.
"""

import argparse
import dataclasses
import time

import numpy as np
import torch

import ddl_amd
from ddl_amd.models.datasets import DummyDataset


class PointCloudProducer(ddl_amd.ProducerFunctionSkeleton):
    """Tabular shard split into (parameters | coordinates+targets | weight) column groups."""

    def __init__(self, n_timesteps, instance, n_instances):
        super().__init__()
        self.n_timesteps, self.instance, self.n_instances = n_timesteps, instance, n_instances
        self.groups = None

    def on_init(self, *args, **kwargs):
        super().on_init(*args, **kwargs)
        ds = DummyDataset(self.n_timesteps, self.instance, self.n_instances,
                          seed=[self.instance, self.producer_index])
        self.groups = [ds.data[:, :3], ds.data[:, 3:8], ds.sample_weight.reshape(-1, 1)]
        n = ds.data.shape[0]
        widths = tuple(g.shape[1] for g in self.groups)
        return ddl_amd.DataProducerOnInitReturn(n, sum(widths), (n, sum(widths)), widths)

    def post_init(self, *args, **kwargs):
        super().post_init(*args, **kwargs)
        self.my_ary[...] = np.hstack(self.groups).astype(np.float32)
        self.groups = None

    def execute_function(self, *args, **kwargs):
        pass  # data are static; the permutation is applied on the device


@dataclasses.dataclass
class Params:
    nepoch: int = 3
    batch_size: int = 64 * 64
    nData: int = 10  # noqa: N815  (timesteps, reference naming)
    fraction_exchange: float = 0.5


@ddl_amd.distributed_dataloader(n_producers=3)
def main(cfg: Params, env, conn):
    producer = PointCloudProducer(cfg.nData, env.rank, env.world_size)
    loader = ddl_amd.DistributedDataLoader(producer, cfg.batch_size, conn, cfg.nepoch, cfg.fraction_exchange,
                                           "alltoall", env.rank, env.world_size, env=env,
                                           order=ddl_amd.OrderSpec(shuffle="device"))
    model = torch.nn.Linear(3, 5).to(loader.device)
    opt = torch.optim.SGD(model.parameters(), lr=1e-2)
    t0 = time.time()
    n = 0
    for epoch in range(cfg.nepoch):
        for i, (pos, target, weight) in enumerate(loader):
            loss = (weight * (model(pos) - target) ** 2).mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            n += pos.shape[0]
            loader.mark(ddl_amd.Marker.END_OF_BATCH)
        loader.mark(ddl_amd.Marker.END_OF_EPOCH)
        if env.rank == 0:
            print(f"epoch {epoch + 1}/{cfg.nepoch}: {len(loader)} batches, loss {loss.item():.4f}", flush=True)
    if env.rank == 0:
        print(f"Training finished: {n} samples/rank in {time.time() - t0:.2f}s on {loader.device}", flush=True)
    return n


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--timesteps", type=int, default=10)
    a = ap.parse_args()
    main(Params(nepoch=a.epochs, nData=a.timesteps))
