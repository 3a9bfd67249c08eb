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
spawned processes, and a process must never be spawned from a GPU-initialised parent (a loader
created after that runs its workers as threads of the process, with a warning).

Every loader alive in a process shares one launcher session (``_Session``): a training loader and an
evaluation loader are opened the usual way, one after the other, and the process groups, the job
watchdog and the death watch live until the LAST loader closes -- closing the training loader leaves
a DDP model built on the group, and the evaluation loader, working.

Mirrors the reference's drop-in entry (``ddl/mpi_dataloader.py:107-249``: ``len``, indexing,
iteration) for users who start from a torch ``Dataset`` rather than a producer function.
"""

from __future__ import annotations

import copy
from typing import Any, Iterator

from .utils.logging import logger


class _Session:
    """The launcher context that every ``DataLoader`` alive in this process shares: the rank's environment,
    the process groups, the job watchdog and the death watch (``parallel.launcher.start``), opened by the
    first loader and closed with the last one. A training loader and an evaluation loader of one program are
    two loaders of ONE session: closing the first leaves the process groups (and a DDP model built on them)
    and the job-wide abort in place for the second."""

    current: "_Session | None" = None

    def __init__(self, cm, env, first_conn):
        self.cm, self.env, self.first_conn = cm, env, first_conn
        self.refs = 0

    @classmethod
    def acquire(cls, num_workers: int, device: str | None):
        """(session, this loader's producer connection)."""
        from .parallel.launcher import spawn_producers, start

        s = cls.current
        if s is None:
            cm = start(n_producers=num_workers, device=device)
            env, conn = cm.__enter__()
            s = cls.current = cls(cm, env, conn)
        else:
            if device is not None and str(device) != s.env.device:
                raise ValueError(f"a DataLoader on {device!r} while the process's loaders run on {s.env.device!r}")
            mode = None
            import torch

            if torch.cuda.is_initialized():
                # a process must never be spawned from a GPU-initialised parent: this loader's workers run as
                # threads of this process (construct every loader before the first CUDA call for processes)
                logger.warning("DataLoader created after the GPU was initialised: its %d workers run as threads",
                               num_workers)
                mode = "thread"
            env = copy.copy(s.env)
            env.n_producers = int(num_workers)
            conn = spawn_producers(env, mode=mode)
            # the session's job abort stops these producers too (start() kills the first connection's spares)
            s.first_conn.spares.append(conn)
        s.refs += 1
        return s, conn

    def release(self, conn) -> None:
        try:
            conn.finalize()
            if conn is not self.first_conn and conn in self.first_conn.spares:
                self.first_conn.spares.remove(conn)
        finally:
            self.refs -= 1
            if self.refs == 0:
                type(self).current = None
                self.cm.__exit__(None, None, None)


class DataLoader:
    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, drop_last: bool = False,
                 num_workers: int = 3, seed: int = 0, epochs: int | None = None, device: str | None = None,
                 resume_state: dict | None = None, host_threads: int = 2, **loader_kw: Any):
        from .dataloader import DistributedDataLoader
        from .models.datasets import MapDatasetSource
        from .models.producers import IndexedProducer

        if num_workers < 1:
            raise ValueError("num_workers must be >= 1 (producer processes fill the pinned windows)")
        self._session, self._conn = _Session.acquire(int(num_workers), device)
        self.env = self._session.env
        try:
            gb = int(batch_size) * self.env.world_size
            producer = IndexedProducer(MapDatasetSource(dataset), gb, seed=int(seed), drop_last=drop_last,
                                       host_threads=host_threads, shuffle=shuffle)
            self.loader = DistributedDataLoader(
                producer, int(batch_size), self._conn, epochs if epochs is not None else 1_000_000, mode="indexed",
                env=self.env, auto_mark=True, seed=int(seed), resume_state=resume_state, **loader_kw)
        except BaseException:
            self._session.release(self._conn)
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
            self._session.release(self._conn)

    def __enter__(self) -> "DataLoader":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
