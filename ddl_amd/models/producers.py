"""Built-in producer functions (``ProducerFunctionSkeleton`` subclasses).

* ``PointwiseProducer``  -- the reference harness's producer (reference
  tests/run_ddl.py:107-167): tabular shard, column groups (3, 5, 1), optional
  host-side row shuffle per round: the pristine shard permuted by the RNG of
  (seed, rank, producer, round), so a window is a function of its round and a
  resumed run reproduces it (at any slot count).
* ``ImageWindowProducer`` -- a window of synthetic 3x224x224 images (bf16 or
  uint8, CHW or HWC). ``execute_function`` stamps the round into every sample
  (a cheap refill that makes each window visit distinct) or regenerates it.
* ``IndexedProducer``    -- world-size-invariant global order: window = one
  rank-local batch of the global batch ``g`` of the ``EpochOrder``; the
  producer gathers the samples out of a node-shared source with the native
  multi-threaded gather straight into its pinned slot.
"""

from __future__ import annotations

import math
from typing import Any

import numpy as np
import torch

from .. import ops
from ..datapusher import DataProducerOnInitReturn
from ..datasetwrapper import ProducerFunctionSkeleton
from ..ops import _dtypes
from ..permutation import EpochOrder, ids_digest
from .datasets import DummyDataset, synthetic_images


class PointwiseProducer(ProducerFunctionSkeleton):
    def __init__(self, n_timesteps: int = 10, idx: int = 0, n_instances: int = 1, host_shuffle: bool = True,
                 seed: int = 0, rows_per_timestep: int | None = None):
        super().__init__()
        self.n_timesteps = n_timesteps
        self.idx = idx
        self.n_instances = n_instances
        self.host_shuffle = host_shuffle
        self.seed = seed
        self.rows_per_timestep = rows_per_timestep
        self.nData = None
        self._groups = None

    def on_init(self, *args, **kwargs):
        super().on_init(*args, **kwargs)
        if self.rows_per_timestep is not None:
            DummyDataset.ROWS_PER_TIMESTEP = self.rows_per_timestep
        ds = DummyDataset(self.n_timesteps, self.idx, self.n_instances,
                          seed=[self.seed, self.rank_global or 0, self.producer_index or 0])
        data, w = ds.data, ds.sample_weight
        self._groups = (data[:, :3], data[:, 3:8], w.reshape(-1, 1))
        self.nData = data.shape[0]
        splits = tuple(g.shape[1] for g in self._groups)
        return DataProducerOnInitReturn(self.nData, sum(splits), (self.nData, sum(splits)), splits, "float32")

    def post_init(self, *args, **kwargs):
        super().post_init(*args, **kwargs)
        # K2 window fill on the native host pool (tests/run_ddl.py:156-159 does np.concatenate)
        ops.pack_columns([torch.from_numpy(np.ascontiguousarray(g, dtype=np.float32)) for g in self._groups],
                         out=torch.from_numpy(self.my_ary))
        self._groups = None
        self._base = self.my_ary.copy() if self.host_shuffle else None

    def execute_function(self, *args, **kwargs):
        """Round r's window = the shard permuted by the RNG of (seed, rank, producer, r).

        The reference shuffles the window in place, round after round (tests/run_ddl.py:163-167),
        so its content depends on every earlier round and on which slot it lands in. Permuting a
        pristine copy instead makes each window a function of its round only: a checkpoint
        resumes it exactly, at any slot count.
        """
        if not self.host_shuffle:
            return
        rng = np.random.default_rng([self.seed, self.rank_global or 0, self.producer_index or 0,
                                     int(kwargs.get("round", 0))])
        np.take(self._base, rng.permutation(len(self._base)), axis=0, out=self.my_ary)


class ImageWindowProducer(ProducerFunctionSkeleton):
    """Synthetic image windows. ``refill`` -- what a producer round does to its slot:

    * ``"stamp"``: writes the round into one element per sample (cheap, distinct windows);
    * ``"full"``: rewrites EVERY byte, as the reference's producers do (``rng.shuffle`` of the whole
      window every round, reference tests/run_ddl.py:163-167): the window is the pristine round-0
      content permuted by the RNG of (seed, rank, producer, round), gathered row by row with the native
      host pool (``host_threads`` threads) -- a function of the round, so resume stays exact;
    * ``"regenerate"``: draws fresh random images (slow: torch RNG on one thread);
    * ``"none"``: leaves the slot as it is.
    """

    def __init__(self, n_samples: int, shape=(3, 224, 224), dtype: Any = "bfloat16", seed: int = 0,
                 refill: str = "stamp", host_threads: int | None = None):
        super().__init__()
        if refill not in ("stamp", "none", "regenerate", "full"):
            raise ValueError("refill must be 'stamp', 'full', 'none' or 'regenerate'")
        self.n_samples = int(n_samples)
        self.shape = tuple(shape)
        self.dtype = dtype
        self.seed = seed
        self.refill = refill
        # a full refill rewrites 77 MB per round: 8 host threads and 2 slots hold the link (53.7 GB/s vs
        # 42.5 GB/s with 4 threads and one slot, archive/profiles/r3_full_refill)
        self.host_threads = int(host_threads) if host_threads is not None else (8 if refill == "full" else 4)
        self.preferred_slots = 2 if refill == "full" else 1
        self._base: torch.Tensor | None = None

    def on_init(self, *args, **kwargs):
        super().on_init(*args, **kwargs)
        nv = int(math.prod(self.shape))
        return DataProducerOnInitReturn(self.n_samples, nv, (self.n_samples, *self.shape), (nv,), self.dtype)

    def _fill(self, t: torch.Tensor, rnd: int) -> None:
        dt = _dtypes.to_torch_dtype(self.dtype)
        s = self.seed * 7919 + (self.rank_global or 0) * 131 + (self.producer_index or 0)
        chunk = 256
        for i in range(0, self.n_samples, chunk):
            n = min(chunk, self.n_samples - i)
            t[i:i + n].copy_(synthetic_images(n, self.shape, dt, seed=s, start=i + rnd * self.n_samples))

    def post_init(self, *args, **kwargs):
        super().post_init(*args, **kwargs)
        self._fill(self.my_tensor, 0)
        if self.refill == "full":
            self._base = self.my_tensor.clone()

    def execute_function(self, *args, **kwargs):
        rnd = int(kwargs.get("round", 0))
        t = kwargs.get("my_tensor", self.my_tensor)
        if self.refill == "stamp":
            flat = t.view(self.n_samples, -1)
            flat[:, 0] = float(rnd % 251) if t.dtype != torch.uint8 else rnd % 251
        elif self.refill == "full":
            from .. import _native

            rng = np.random.default_rng([self.seed, self.rank_global or 0, self.producer_index or 0, rnd])
            base = self._base
            _native.runtime().gather_rows(t.data_ptr(), base.data_ptr(), base[0].numel() * base.element_size(),
                                          rng.permutation(self.n_samples).astype(np.int64), self.n_samples,
                                          self.host_threads)
        elif self.refill == "regenerate":
            self._fill(t, rnd)


class IndexedProducer(ProducerFunctionSkeleton):
    """Producer of the world-size-invariant global order (one window = one local batch)."""

    def __init__(self, source, global_batch: int, seed: int | None = None, drop_last: bool = True,
                 host_threads: int = 4, shuffle: bool = True, worker_init_fn=None):
        super().__init__()
        self.source = source
        self.worker_init_fn = worker_init_fn  # torch's: called with the worker (producer) index in the worker
        self.global_batch = int(global_batch)
        self.seed = seed  # None: use the loader's seed
        self.drop_last = drop_last
        self.shuffle = bool(shuffle)  # False: dataset order (evaluation)
        self.host_threads = host_threads
        self.world_size = 1
        self.order: EpochOrder | None = None

    def on_init(self, *args, **kwargs):
        super().on_init(*args, **kwargs)
        self.world_size = int(kwargs.get("world_size", 1))
        init_fn = getattr(self, "worker_init_fn", None)
        if init_fn is not None:
            init_fn(int(self.producer_index or 0))
        if self.seed is None:
            self.seed = int(kwargs.get("seed", 0))
        self.order = EpochOrder(self.source.n, self.global_batch, int(self.seed), self.drop_last, self.shuffle)
        lb = self.order.local_batch(self.world_size)
        nv = int(math.prod(self.source.sample_shape)) if self.source.sample_shape else 1
        return DataProducerOnInitReturn(lb, nv, (lb, *self.source.sample_shape), (nv,), self.source.dtype,
                                        extra={"batches_per_epoch": self.order.batches_per_epoch,
                                               "global_batch": self.global_batch, "n_samples": self.source.n,
                                               "order_seed": int(self.seed), "order_shuffle": self.shuffle,
                                               "order_drop_last": self.drop_last,
                                               # MapDatasetSource: the loader rebuilds the sample structure
                                               "fields": getattr(self.source, "fields", None),
                                               "fields_kind": getattr(self.source, "kind", None)})

    def post_init(self, *args, **kwargs):
        super().post_init(*args, **kwargs)

    def batch_position(self, rnd: int) -> tuple[int, int]:
        """(epoch, global batch) this producer delivers in round ``rnd``."""
        assert self.order is not None
        g_total = rnd * (self.n_producers or 1) + (self.producer_index or 0)
        return divmod(g_total, self.order.batches_per_epoch)

    def batch_indices(self, rnd: int) -> np.ndarray:
        epoch, g = self.batch_position(rnd)
        return self.order.indices(epoch, g, self.rank_global or 0, self.world_size)

    def execute_function(self, *args, **kwargs):
        rnd = int(kwargs.get("round", 0))
        t: torch.Tensor = kwargs.get("my_tensor", self.my_tensor)
        epoch, g = self.batch_position(rnd)
        idx = self.order.indices(epoch, g, self.rank_global or 0, self.world_size)
        self.source.gather(idx, t.data_ptr(), self.host_threads)
        # slot tags: which batch this window is, and a digest of its sample ids (verify_order)
        return {"tags": [epoch, g, ids_digest(idx)]}
