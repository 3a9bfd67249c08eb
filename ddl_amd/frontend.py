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
yields a shorter last batch). ``drop_last=True`` drops the partial batch. The workers are processes,
as with torch's DataLoader at ``num_workers > 0``; they are started with the ``spawn`` method (a fresh
interpreter, not a ``fork`` that would inherit this process's HIP context), so a loader may be created
before or after the process first touches the GPU.

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
    def acquire(cls, num_workers: int, device: str | None, mode: str | None = None):
        """(session, this loader's producer connection); ``mode``: the workers' mode (spawn_producers)."""
        from .parallel.launcher import spawn_producers, start

        s = cls.current
        if s is None:
            cm = start(n_producers=num_workers, device=device, producer_mode=mode)
            env, conn = cm.__enter__()
            s = cls.current = cls(cm, env, conn)
        else:
            if device is not None and str(device) != s.env.device:
                raise ValueError(f"a DataLoader on {device!r} while the process's loaders run on {s.env.device!r}")
            env = copy.copy(s.env)
            env.n_producers = int(num_workers)
            # "spawn" start method: each worker is a fresh interpreter (fork + exec), never a fork that inherits
            # this process's HIP context, so a loader created after the GPU is in use is fine
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
    """``torch.utils.data.DataLoader(dataset, ...)`` with torch's signature; see the module docstring.

    torch's arguments and what they mean here:

    * ``batch_size``, ``shuffle``, ``drop_last``: as in torch (``batch_size`` per rank, see above);
    * ``num_workers``: producer worker processes of this rank; ``0`` (torch: load in the main process) runs
      one worker as a thread of this process;
    * ``timeout``: > 0 bounds every wait of the loader (``timeout_s``); 0 keeps the loader's own default bound
      (the loader never waits forever);
    * ``worker_init_fn(worker_id)``: called in each worker before its first sample (picklable, as under
      torch's ``spawn`` workers);
    * ``generator``: the order's seed when ``seed`` is not given (``generator.initial_seed()``);
    * ``pin_memory``, ``pin_memory_device``, ``persistent_workers``, ``prefetch_factor``,
      ``multiprocessing_context``: accepted; batches land in HBM from pinned windows, the workers live as
      long as the loader, windows are prefetched ``prefetch_depth`` ahead, workers are always ``spawn``ed;
    * ``sampler``, ``batch_sampler``, a ``collate_fn`` other than ``default_collate``, ``in_order=False``:
      rejected with a ``ValueError`` -- the order is the world-size-invariant ``EpochOrder`` (``shuffle``,
      ``seed``) and batches are assembled on the device from the sample's fields, as ``default_collate``
      would stack them.
    """

    def __init__(self, dataset, batch_size: int | None = 1, shuffle: bool | None = None, sampler=None,
                 batch_sampler=None, num_workers: int = 3, collate_fn=None, pin_memory: bool = True,
                 drop_last: bool = False, timeout: float = 0, worker_init_fn=None, multiprocessing_context=None,
                 generator=None, *, prefetch_factor: int | None = None, persistent_workers: bool = True,
                 pin_memory_device: str = "", in_order: bool = True, seed: int | None = None,
                 epochs: int | None = None, device: str | None = None, resume_state: dict | None = None,
                 host_threads: int = 2, **loader_kw: Any):
        import torch

        from .dataloader import DistributedDataLoader
        from .models.datasets import MapDatasetSource
        from .specs import from_flat
        from .models.producers import IndexedProducer

        if sampler is not None or batch_sampler is not None:
            raise ValueError("ddl_amd.DataLoader has no sampler / batch_sampler: the order is the world-size-"
                             "invariant EpochOrder (shuffle=, seed=), already split across ranks like a "
                             "DistributedSampler")
        if collate_fn is not None and collate_fn is not torch.utils.data.default_collate:
            raise ValueError("ddl_amd.DataLoader assembles batches on the device as default_collate stacks them; "
                             "a custom collate_fn is not supported (return the collated fields from __getitem__)")
        if not in_order:
            raise ValueError("in_order=False is not supported: batches always come in the epoch order")
        if batch_size is None or int(batch_size) < 1:
            raise ValueError("batch_size must be a positive integer (batches are assembled by the loader)")
        if isinstance(dataset, torch.utils.data.IterableDataset) or not hasattr(dataset, "__getitem__"):
            raise TypeError("ddl_amd.DataLoader takes a map-style dataset (len(ds), ds[i]); for a stream of "
                            "samples write a producer (ddl_amd.ProducerFunctionSkeleton)")
        if int(num_workers) < 0:
            raise ValueError("num_workers must be >= 0")
        if seed is None:
            seed = int(generator.initial_seed()) % (1 << 63) if generator is not None else 0
        if timeout and float(timeout) > 0:
            loader_kw.setdefault("timeout_s", float(timeout))
        # num_workers=0: torch loads in the main process; here one worker thread of this process
        n_workers, mode = (int(num_workers), None) if int(num_workers) > 0 else (1, "thread")
        self._session, self._conn = _Session.acquire(n_workers, device, mode)
        self.env = self._session.env
        try:
            gb = int(batch_size) * self.env.world_size
            producer = IndexedProducer(MapDatasetSource(dataset), gb, seed=int(seed), drop_last=drop_last,
                                       host_threads=host_threads, shuffle=bool(shuffle),
                                       worker_init_fn=worker_init_fn)
            specs = from_flat(loader_kw, mode="indexed", seed=int(seed))
            self.loader = DistributedDataLoader(
                producer, int(batch_size), self._conn, epochs if epochs is not None else 1_000_000, env=self.env,
                auto_mark=True, resume_state=resume_state, **specs, **loader_kw)
        except BaseException:
            self._session.release(self._conn)
            raise
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.num_workers = int(num_workers)
        self.drop_last = bool(drop_last)
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
