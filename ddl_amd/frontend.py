"""A ``torch.utils.data.DataLoader``-shaped front end over the ddl_amd machinery.

    loader = ddl_amd.DataLoader(dataset, batch_size=256, shuffle=True, num_workers=3, seed=0)
    for epoch in range(10):
        loader.set_epoch(epoch)          # optional: the loader also advances by itself
        for images, labels in loader:    # device tensors, the dataset's sample structure
            ...
    torch.save(loader.state_dict(), ...)   # epoch / global-batch (sample-index) cursor

What it wires together, each piece usable on its own:

* ``ddl_amd.start`` -- the rank's environment (torchrun / SLURM variables, RCCL DP group) and
  ``num_workers`` producer processes, spawned before this process touches the GPU;
* ``MapDatasetSource`` + ``IndexedProducer`` -- producers call ``dataset[i]`` for their share of every
  global batch of the world-size-invariant ``EpochOrder`` and pack the samples into pinned windows;
* ``DistributedDataLoader(mode="indexed", auto_mark=True)`` -- native staging into HBM and
  per-batch dispatch; batches come back as typed views in the sample's structure.

``batch_size`` is the per-rank batch, as with ``DistributedSampler`` under DDP: the global batch is
``batch_size * world_size``, and rank r gets slice r of every global batch. ``drop_last`` defaults to
False as in torch: no sample of the epoch is dropped. Every batch is full (static shapes): the last,
partial global batch is completed from the start of the epoch's order, which is what
``DistributedSampler(drop_last=False)`` does under DDP (torch's single-process DataLoader instead
yields a shorter last batch). ``drop_last=True`` drops the partial batch. Like torch's DataLoader
with worker processes, construct it before the first CUDA call of the process: the workers are
spawned processes (on a box whose policy forbids spawning after GPU initialisation, that ordering
is required).

Mirrors the reference's drop-in entry (``ddl/mpi_dataloader.py:107-249``: ``len``, indexing,
iteration) for users who start from a torch ``Dataset`` rather than a producer function.
"""

from __future__ import annotations

from typing import Any, Iterator


class DataLoader:
    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, drop_last: bool = False,
                 num_workers: int = 3, seed: int = 0, epochs: int | None = None, device: str | None = None,
                 resume_state: dict | None = None, host_threads: int = 2, **loader_kw: Any):
        from .dataloader import DistributedDataLoader
        from .models.datasets import MapDatasetSource
        from .models.producers import IndexedProducer
        from .parallel.launcher import start

        if num_workers < 1:
            raise ValueError("num_workers must be >= 1 (producer processes fill the pinned windows)")
        self._cm = start(n_producers=int(num_workers), device=device)
        self.env, conn = self._cm.__enter__()
        try:
            gb = int(batch_size) * self.env.world_size
            producer = IndexedProducer(MapDatasetSource(dataset), gb, seed=int(seed), drop_last=drop_last,
                                       host_threads=host_threads, shuffle=shuffle)
            self.loader = DistributedDataLoader(
                producer, int(batch_size), conn, epochs if epochs is not None else 1_000_000, mode="indexed",
                env=self.env, auto_mark=True, seed=int(seed), resume_state=resume_state, **loader_kw)
        except BaseException:
            self._cm.__exit__(None, None, None)
            raise
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self._closed = False

    # torch DataLoader surface ---------------------------------------------------------------
    def __iter__(self) -> Iterator:
        """One epoch (the rest of it after a resume); the next ``iter()`` continues with the next epoch."""
        return iter(self.loader)

    def __len__(self) -> int:
        return len(self.loader)

    def set_epoch(self, epoch: int) -> None:
        self.loader.set_epoch(epoch)

    def state_dict(self) -> dict:
        return self.loader.state_dict()

    def load_state_dict(self, sd: dict) -> None:
        self.loader.load_state_dict(sd)

    def stats(self) -> dict:
        return self.loader.stats()

    # lifetime ------------------------------------------------------------------------------
    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        try:
            self.loader.close()
        finally:
            self._cm.__exit__(None, None, None)

    def __enter__(self) -> "DataLoader":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
