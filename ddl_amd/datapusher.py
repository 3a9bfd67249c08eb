"""Producer engine ("data pusher", reference ddl/datapusher.py:14-170).

Runs in a producer worker process (a child of the consumer, never touching the
GPU). Lifecycle, as in the reference:

1. receive the consumer's metadata (incl. the pickled user producer function);
2. ``on_init`` -> ``DataProducerOnInitReturn`` (window geometry);
3. send window metadata back; attach the shm arena; ``post_init`` fills slot 0
   (replicated into the other slots with the native parallel copy);
4. barrier; then the hot loop: wait for a free slot -> ``global_shuffle`` /
   ``execute_function`` hooks refill it in place -> publish -> next slot;
5. stop on the shutdown word; ``on_push_end``.

Differences from the reference: every registered hook runs (the reference
dispatches only ``callbacks[0]``, ddl/utils.py:22), windows may be any dtype
(reference f32 only, ddl/connection.py:105), ``n_slots`` windows per producer
let the producer refill one while the consumer still holds another, and
failures are reported to the consumer instead of hanging it.
"""

from __future__ import annotations

import dataclasses
import math
import os
import time
from abc import ABC, abstractmethod
from typing import Any

import numpy as np
import torch

from .connection import ProducerConnection
from .exceptions import ShapeMismatchError, ShutdownError
from .ops import _dtypes
from .types import MetaData_Consumer_To_Producer, MetaData_Producer_To_Consumer, WorkerInfo
from .utils import faults
from .utils.callbacks import execute_callbacks
from .utils.logging import for_all_methods, logger, set_role, with_logging


@dataclasses.dataclass
class DataProducerOnInitReturn:
    """What ``on_init`` returns (reference ddl/datapusher.py:14-19) + ``dtype``.

    ``shape`` is ``(nData, *sample_shape)``; ``nValues`` = prod(sample_shape);
    ``splits`` partitions the flattened sample into column groups (the batch
    is returned as one tensor per group).
    """

    nData: int  # noqa: N815
    nValues: int  # noqa: N815
    shape: tuple[int, ...]
    splits: tuple[int, ...]
    dtype: Any = "float32"
    extra: dict = dataclasses.field(default_factory=dict)  # forwarded to the consumer (e.g. batches_per_epoch)

    def validate(self) -> None:
        if self.nData <= 0 or self.nValues <= 0:
            raise ShapeMismatchError((self.nData, self.nValues), "nData and nValues must be positive")
        if not self.shape or self.shape[0] != self.nData:
            raise ShapeMismatchError(self.shape, f"shape[0] must equal nData={self.nData}")
        if math.prod(self.shape[1:]) != self.nValues:
            raise ShapeMismatchError(self.shape, f"prod(shape[1:]) must equal nValues={self.nValues}")
        if sum(self.splits) != self.nValues:
            raise ShapeMismatchError(self.splits, f"splits must sum to nValues={self.nValues}")


class DataPusherABC(ABC):
    """The reference's abstract producer engine (ddl/datapusher.py:22-41)."""

    @abstractmethod
    def push_data(self) -> None: ...

    @abstractmethod
    def _start_access_epoch(self, target_rank: int = -1) -> None: ...

    @abstractmethod
    def _end_access_epoch(self, target_rank: int = -1) -> None: ...

    @abstractmethod
    def sync(self) -> None: ...

    @abstractmethod
    def _finalize(self) -> None: ...


@for_all_methods(with_logging, exclude=["_fill_round", "_istart_access_epoch", "_iend_access_epoch", "sync"])
class DataPusher(DataPusherABC):
    def __init__(self, connection: ProducerConnection, rank_global: int = 0, world_size: int = 1):
        self.connection = connection
        self.rank_global = rank_global
        self.world_size = world_size
        self.callbacks: list[Any] = []

        meta: MetaData_Consumer_To_Producer = connection.recv_metadata_as_producer()
        self.meta = meta
        self.index = meta.producer_index
        set_role("producer", self.index)
        self.callbacks.append(meta.producer_function)

        ret = execute_callbacks(
            "on_init", self.callbacks, rank_global=rank_global, producer_index=self.index,
            n_producers=meta.n_producers, world_size=world_size, seed=meta.seed)
        if not isinstance(ret, DataProducerOnInitReturn):
            raise TypeError(f"on_init must return DataProducerOnInitReturn, got {type(ret).__name__}")
        ret.validate()
        self.init_ret = ret
        self.dtype = _dtypes.to_torch_dtype(ret.dtype)
        bpw = ret.nData // meta.batch_size
        if bpw <= 0:
            raise ShapeMismatchError((ret.nData, meta.batch_size),
                                     f"window of {ret.nData} samples holds no batch of {meta.batch_size}")
        self.metadata_to_consumer = MetaData_Producer_To_Consumer(
            nData=ret.nData, nValues=ret.nValues, shape=tuple(ret.shape), splits=tuple(ret.splits),
            batches_per_window=bpw, dtype=str(self.dtype).replace("torch.", ""), pid=os.getpid(),
            extra=dict(ret.extra))
        connection.send_metadata(self.metadata_to_consumer, "producer")

        self.views = connection.attach_windows(tuple(ret.shape), self.dtype)
        self.window_bytes = int(math.prod(ret.shape)) * _dtypes.itemsize(self.dtype)
        my_ary, my_tensor = self.views[0]
        self._set_user_window(my_ary, my_tensor)
        execute_callbacks("post_init", self.callbacks, rank_global=rank_global, my_ary=my_ary, my_tensor=my_tensor,
                          n_instance=world_size, producer_index=self.index)
        self._replicate_slot0()
        connection.Barrier()

    def _set_user_window(self, my_ary, my_tensor) -> None:
        for cb in self.callbacks:
            if hasattr(cb, "my_ary"):
                cb.my_ary = my_ary
            if hasattr(cb, "my_tensor"):
                cb.my_tensor = my_tensor

    def _replicate_slot0(self) -> None:
        n_slots = len(self.views)
        if n_slots <= 1:
            return
        from . import _native

        rt = _native.runtime()
        src = self.connection.arena.slot_address(self.index, 0)
        for s in range(1, n_slots):
            rt.parallel_copy(self.connection.arena.slot_address(self.index, s), src, self.window_bytes,
                             self.meta.host_threads)

    def _fill_round(self, slot: int, rnd: int) -> None:
        my_ary, my_tensor = self.views[slot]
        self._set_user_window(my_ary, my_tensor)
        kw = dict(my_ary=my_ary, my_tensor=my_tensor, round=rnd, slot=slot, producer_index=self.index)
        execute_callbacks("global_shuffle", self.callbacks, **kw)
        ret = execute_callbacks("execute_function", self.callbacks, **kw)
        # optional publish metadata: a list of <=4 ints (slot tags) or
        # {"tags": [...], "used_bytes": n} (ship only the first n bytes H2D)
        if isinstance(ret, dict):
            return list(ret.get("tags", [])), int(ret.get("used_bytes", self.window_bytes))
        if isinstance(ret, (list, tuple)) and all(isinstance(x, (int, np.integer)) for x in ret):
            return [int(x) for x in ret], self.window_bytes
        return [], self.window_bytes

    # ------------------------------------------------- reference protocol names
    def sync(self) -> None:
        """The reference's ``Win.Sync`` barrier (ddl/datapusher.py:126-127). Here the
        slot state word is stored with release / loaded with acquire semantics
        around every hand-off, which orders the window bytes: nothing to do."""

    def _start_access_epoch(self, target_rank: int = -1) -> None:
        """No-op, as in the reference (ddl/datapusher.py:129-130)."""

    def _end_access_epoch(self, target_rank: int = -1) -> None:
        """No-op, as in the reference (ddl/datapusher.py:132-133)."""

    def _istart_access_epoch(self, slot: int) -> WorkerInfo:
        """Wait until the consumer hands ``slot`` back, or shutdown (ddl/datapusher.py:135-136)."""
        return self.connection.Istart_access_epoch(slot)

    def _iend_access_epoch(self, slot: int, rnd: int, used: int, tags: list) -> WorkerInfo:
        """Publish ``slot`` to the consumer (ddl/datapusher.py:138-139)."""
        return self.connection.Iend_access_epoch(slot, seq=rnd, used_bytes=used, epoch=rnd, tags=tags)

    def _finalize(self) -> None:
        self.connection.finalize()

    def push_data(self) -> None:
        """Hot loop (reference ddl/datapusher.py:147-170)."""
        conn = self.connection
        n_slots = len(self.views)
        execute_callbacks("on_push_begin", self.callbacks)
        rnd = self.meta.start_round
        slot = rnd % n_slots
        while True:
            ctl = conn.poll_control()
            if ctl is not None:
                if ctl[0] != "seek":
                    raise RuntimeError(f"producer {self.index}: unexpected control message {ctl[0]!r}")
                rnd = conn.pause_for_seek()  # live load_state_dict / set_epoch on the consumer
                slot = rnd % n_slots
                continue
            t0 = time.perf_counter_ns()
            if self._istart_access_epoch(slot) is WorkerInfo.STOP:
                break
            t1 = time.perf_counter_ns()
            faults.maybe_fail_producer(self.index, rnd)
            self.sync()
            tags, used = self._fill_round(slot, rnd)
            t2 = time.perf_counter_ns()
            if self._iend_access_epoch(slot, rnd, used, tags) is WorkerInfo.STOP:
                break
            conn.arena.heartbeat(self.index, t2 - t1, t1 - t0)
            execute_callbacks("on_shuffle_end", self.callbacks, round=rnd, slot=slot)
            rnd += 1
            slot = (slot + 1) % n_slots
        execute_callbacks("on_push_end", self.callbacks)
        self._finalize()


def producer_main(pipe, producer_index: int, consumer_pid: int, rank: int, world_size: int,
                  timeout_s: float, env_overrides: dict | None = None, in_thread: bool = False) -> None:
    """Entry point of a producer worker (spawned process, or thread of the consumer)."""
    if not in_thread:
        if env_overrides:
            os.environ.update(env_overrides)
        # Producers are host-only: make sure nothing in them can grab the GPU.
        os.environ["HIP_VISIBLE_DEVICES"] = "-1"  # producers never touch a GPU
        torch.set_num_threads(1)  # heavy host work runs on the native gather pools, not torch's
    set_role("producer", producer_index)
    from .utils.logging import configure

    configure()
    conn = ProducerConnection(pipe, producer_index, consumer_pid, timeout_s)
    try:
        pusher = DataPusher(conn, rank_global=rank, world_size=world_size)
        pusher.push_data()
        del pusher
    except ShutdownError:  # closed before any loader used this producer (e.g. an unused spare connection)
        logger.debug("producer %d: shut down before a loader used it", producer_index)
    except BaseException as e:  # report, then exit non-zero
        logger.error("producer %d failed: %r", producer_index, e)
        conn.report_error(e)
        if not in_thread:
            raise SystemExit(1)
    if not in_thread:
        _exit_quickly()


def _exit_quickly() -> None:
    """End a producer process after its clean shutdown without the interpreter teardown: with torch loaded
    that teardown (module and C++ static destructors) took ~0.8 s, which the consumer waited out at the end of
    its last epoch (``connection.finalize`` joins the producers). The producer object has been released
    already (its ``__del__``, and its files' close and flush, ran), and the ``atexit`` handlers run first
    (logging flushes, the user's own handlers)."""
    import atexit
    import sys

    atexit._run_exitfuncs()
    for f in (sys.stdout, sys.stderr):
        try:
            f.flush()
        except Exception:  # pragma: no cover - a closed stream
            pass
    os._exit(0)
