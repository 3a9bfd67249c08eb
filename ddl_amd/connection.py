"""Consumer <-> producer transport of one GPU group (reference ddl/connection.py).

Reference mechanism -> this implementation:

* MPI-3 ``Win.Allocate_shared`` windows, one collective per producer, f32 only
  (reference ddl/connection.py:88-139)  ->  ONE native shm arena per GPU group
  (``csrc/runtime/arena.cpp``), any dtype, ``n_slots`` windows per producer,
  2 MiB-aligned regions; the consumer pins the whole arena with
  ``hipHostRegister`` so H2D copies DMA straight out of it.
* zero-byte tag-7 ``Ssend``/``Recv``/``Issend``/``Irecv`` + ``Win.Sync``
  ownership hand-off (reference ddl/connection.py:153-182)  ->  per-slot
  state word EMPTY -> READY -> HELD -> EMPTY with release/acquire atomics and
  futex wait/wake; the consumer's release can be *enqueued on a HIP stream*
  (``hipLaunchHostFunc``) so a slot returns to its producer the moment its
  H2D copy retires, without the consumer thread.
* ``Ibarrier`` on a ``Dup``'d communicator as the shutdown signal
  (reference ddl/connection.py:32-37,184-187)  ->  the arena's shutdown word;
  every wait is bounded and wakes on shutdown, producer failure or death
  (reference: a dead producer blocks the consumer in ``Recv`` forever).
* pickled ``ssend``/``recv`` of metadata (reference ddl/connection.py:65-86)
  ->  multiprocessing pipes to the spawned producer workers.
"""

from __future__ import annotations

import math
import os
import time
import traceback
import uuid
from typing import Any

import numpy as np
import torch

from . import _native
from .exceptions import DDLTimeoutError, PeerDeathError, ShutdownError
from .ops import _dtypes
from .types import MetaData_Consumer_To_Producer, MetaData_Producer_To_Consumer, WorkerInfo
from .utils.logging import for_all_methods, logger, with_logging

DEFAULT_TIMEOUT_S = float(os.environ.get("DDL_TIMEOUT_S", "600"))


def _window_view(arena, p: int, s: int, shape: tuple[int, ...], dtype: torch.dtype):
    """(numpy-or-torch view, torch view) of slot (p, s) as an array of ``shape``."""
    nbytes = int(math.prod(shape)) * _dtypes.itemsize(dtype)
    mv = arena.slot_view(p, s)
    t = torch.frombuffer(mv, dtype=torch.uint8, count=nbytes).view(dtype).view(shape)
    npd = _dtypes.numpy_view_dtype(dtype)
    if npd is not None:
        a = np.frombuffer(mv, dtype=npd, count=int(math.prod(shape))).reshape(shape)
        return a, t
    return t, t


class _Pipe:
    """Tagged-message helper over a multiprocessing connection with liveness checks."""

    def __init__(self, conn, peer: Any = None, name: str = "peer"):
        self.conn = conn
        self.peer = peer  # multiprocessing.Process (consumer side) or None
        self.name = name

    def send(self, tag: str, payload: Any = None) -> None:
        self.conn.send((tag, payload))

    def recv(self, expect: str, timeout_s: float) -> Any:
        deadline = time.monotonic() + timeout_s
        while True:
            if self.conn.poll(0.05):
                try:
                    tag, payload = self.conn.recv()
                except (EOFError, OSError) as e:
                    raise PeerDeathError(
                        f"{self.name}: connection lost while waiting for {expect!r} ({e!r})") from None
                if tag == "error":
                    raise PeerDeathError(f"{self.name} failed:\n{payload}")
                if tag == "shutdown" and expect != "shutdown":  # the consumer closed before using this producer
                    raise ShutdownError(f"{self.name}: shut down while waiting for {expect!r}")
                if tag != expect:
                    raise RuntimeError(f"{self.name}: protocol error, expected {expect!r} got {tag!r}")
                return payload
            if self.peer is not None and not self.peer.is_alive():
                # drain a final error message if the peer managed to send one
                if self.conn.poll(0):
                    continue
                raise PeerDeathError(f"{self.name} died (exit code {getattr(self.peer, 'exitcode', None)}) while we "
                                     f"waited for {expect!r}", pid=getattr(self.peer, "pid", None))
            if time.monotonic() > deadline:
                raise DDLTimeoutError(f"{self.name}: timed out after {timeout_s:.0f}s waiting for {expect!r}")


def _raise_for(rc, what: str, producer: int | None = None, pid: int | None = None) -> None:
    rt = _native.runtime()
    if rc == rt.WaitResult.OK:
        return
    if rc == rt.WaitResult.SHUTDOWN:
        raise ShutdownError(f"{what}: loader was shut down")
    if rc == rt.WaitResult.TIMEOUT:
        raise DDLTimeoutError(f"{what}: timed out")
    if rc == rt.WaitResult.PEER_FAILED:
        raise PeerDeathError(f"{what}: producer {producer} reported a failure", producer, pid)
    raise PeerDeathError(f"{what}: peer process {pid} died", producer, pid)


@for_all_methods(with_logging, exclude=["acquire", "release", "release_on_stream", "slot_info"])
class Connection:
    """Consumer-side end of the GPU group: owns the arena and the producer pipes."""

    role = "consumer"

    def __init__(self, pipes: list, processes: list | None = None, timeout_s: float = DEFAULT_TIMEOUT_S,
                 rank: int = 0):
        self.n_producers = len(pipes)
        self.timeout_s = timeout_s
        self.rank = rank
        procs = processes or [None] * len(pipes)
        self.pipes = [_Pipe(c, p, f"producer {i}") for i, (c, p) in enumerate(zip(pipes, procs))]
        self.processes = list(procs)
        self.arena = None
        self.cpu_layout: dict | None = None  # consumer / producer CPU split (utils/numa.partition_after_spawn)
        self.spares: list["Connection"] = []  # more producer sets spawned with this one (start(spare_connections=))
        self._finalizers: list = []
        self.window_shapes: list[tuple[int, ...]] = []
        self.window_dtypes: list[torch.dtype] = []
        self.n_slots = 1
        self._registered = False
        self._closed = False

    # ------------------------------------------------------------ metadata
    def send_metadata(self, metadata: MetaData_Consumer_To_Producer, called_from: str = "consumer") -> None:
        if called_from != "consumer":
            raise ValueError(f"{called_from=} is not valid on the consumer side")
        import copy

        for i, p in enumerate(self.pipes):
            m = copy.copy(metadata)
            m.producer_index = i
            m.n_producers = self.n_producers
            p.send("meta", m)

    def recv_metadata_as_consumer(self) -> list[MetaData_Producer_To_Consumer]:
        return [p.recv("meta", self.timeout_s) for p in self.pipes]

    @property
    def producer_pids(self) -> list[int]:
        # producer threads (thread mode) share our pid: liveness = thread liveness via the pipe
        return [getattr(p, "pid", 0) or 0 for p in self.processes]

    # ------------------------------------------------------------- windows
    def init_windows(self, shapes: list[tuple[int, ...]], dtypes: list[torch.dtype], n_slots: int = 1,
                     pin: bool | None = None) -> list[list[tuple[Any, torch.Tensor]]]:
        """Create the arena (one region per producer slot), hand its name to the producers.

        Returns ``views[p][s] = (numpy-or-torch view, torch view)``.
        """
        rt = _native.runtime()
        caps = [int(math.prod(s)) * _dtypes.itemsize(d) for s, d in zip(shapes, dtypes)]
        name = f"/ddl_amd.{os.getpid()}.{self.rank}.{uuid.uuid4().hex[:8]}"
        self.arena = rt.Arena.create(name, caps, n_slots)
        self.window_shapes = [tuple(s) for s in shapes]
        self.window_dtypes = list(dtypes)
        self.n_slots = n_slots
        try:
            for p in self.pipes:
                p.send("arena", name)
            for p in self.pipes:
                p.recv("attached", self.timeout_s)
        finally:
            self.arena.unlink()  # everyone has it mapped (or failed): no /dev/shm leak
        for i, pid in enumerate(self.producer_pids):
            if pid:
                self.arena.set_producer_pid(i, pid)
        if pin is None:
            pin = _native.gpu_available()
        if pin:
            self.pin()
        return [[_window_view(self.arena, p, s, self.window_shapes[p], self.window_dtypes[p]) for s in range(n_slots)]
                for p in range(self.n_producers)]

    def pin(self) -> None:
        """Page-lock + device-map the whole arena (hipHostRegister, mapped)."""
        if self._registered or self.arena is None:
            return
        _native.hip().host_register(self.arena.base_address, self.arena.total_bytes, True)
        self._registered = True

    @property
    def pinned(self) -> bool:
        return self._registered

    def slot_address(self, p: int, s: int) -> int:
        return self.arena.slot_address(p, s)

    def slot_device_address(self, p: int, s: int) -> int:
        base = _native.hip().host_device_pointer(self.arena.base_address)
        return base + (self.arena.slot_address(p, s) - self.arena.base_address)

    def slot_info(self, p: int, s: int) -> dict:
        return self.arena.slot_info(p, s)

    def Barrier(self) -> None:  # noqa: N802  (reference name)
        """Rendezvous with every producer (reference ddl/connection.py:141)."""
        for p in self.pipes:
            p.recv("barrier", self.timeout_s)
        for p in self.pipes:
            p.send("barrier")

    def lock_windows(self) -> None:
        """Reference ``Lock_all`` passive-target epoch (ddl/connection.py:39-43).

        Nothing to do here: slot ownership is the arena's per-slot state word
        (acquire/release atomics + futex), so there is no RMA epoch to open.
        """

    def unlock_windows(self) -> None:
        """Reference ``Unlock_all`` (ddl/connection.py:45-49); see ``lock_windows``."""

    def sync(self, target: int = 0) -> None:
        """Reference ``Win.Sync`` memory barrier (ddl/connection.py:61-63, 144-151).

        Nothing to do: every hand-off stores the slot state word with release and
        loads it with acquire semantics (csrc/runtime/arena.cpp), which orders the
        window bytes; device reads are ordered by the H2D copy's stream events.
        """

    _sync = sync

    # ------------------------------------------------------------ hand-off
    def acquire(self, p: int, s: int, timeout_s: float | None = None) -> dict:
        """Wait until producer ``p`` publishes slot ``s``; take it (READY -> HELD).

        Reference: ``start_access_epoch`` (0-byte Recv tag 7 + Win.Sync,
        ddl/connection.py:153-155).
        """
        rt = _native.runtime()
        t = self.timeout_s if timeout_s is None else timeout_s
        rc = self.arena.wait_state(p, s, rt.READY, int(t * 1000), self.producer_pids[p], p)
        _raise_for(rc, f"acquire(producer {p}, slot {s})", p, self.producer_pids[p])
        self.arena.set_state(p, s, rt.HELD)
        return self.arena.slot_info(p, s)

    def release(self, p: int, s: int) -> None:
        """Hand slot ``s`` back to producer ``p`` now (reference ``end_access_epoch``)."""
        self.arena.set_state(p, s, _native.runtime().EMPTY)

    def seek_producers(self, start_rounds: list[int]) -> None:
        """Reposition every producer to continue at round ``start_rounds[p]`` (live resume).

        The caller has stopped everything that reads the slots (stager thread joined, copies
        retired). Protocol: ``seek`` to each producer; every slot set EMPTY, which wakes a
        producer blocked on a slot (it may publish one stale round, then sees the message at
        the top of its loop); wait for every ``seek_ack`` (each producer is now parked on its
        pipe); discard whatever was published meanwhile (all slots EMPTY again); ``go`` with
        the new round. Nothing runs concurrently with the final reset, so no stale window can
        survive it.
        """
        if len(start_rounds) != self.n_producers:
            raise ValueError("one start round per producer")
        empty = _native.runtime().EMPTY
        for p in self.pipes:
            p.send("seek")
        n_slots = self.arena.n_slots
        for i in range(self.n_producers):
            for s in range(n_slots):
                self.arena.set_state(i, s, empty)
        for p in self.pipes:
            p.recv("seek_ack", self.timeout_s)
        for i in range(self.n_producers):
            for s in range(n_slots):
                self.arena.set_state(i, s, empty)
        for p, r in zip(self.pipes, start_rounds):
            p.send("go", int(r))

    def release_on_stream(self, p: int, s: int, stream) -> None:
        """Hand the slot back when ``stream`` reaches this point (after its H2D copy)."""
        handle = stream if isinstance(stream, int) else stream.cuda_stream
        _native.hip().enqueue_release(self.arena.state_address(p, s), _native.runtime().EMPTY, handle)

    # backwards-compatible names (reference ddl/connection.py:153-159)
    def start_access_epoch(self, target: int, slot: int = 0) -> None:
        self.acquire(target - 1, slot)

    def end_access_epoch(self, target: int, slot: int = 0) -> None:
        self.release(target - 1, slot)

    # ------------------------------------------------------------ shutdown
    def shutdown_operation(self) -> None:
        """Signal every producer to stop (reference: consumer Ibarrier, ddl/connection.py:184-187)."""
        if self.arena is not None:
            self.arena.request_shutdown()
        for p in self.pipes:
            try:
                p.send("shutdown")
            except (BrokenPipeError, OSError):
                pass

    def quarantine(self) -> None:
        """A stager closed with copies out of the arena still pending (a hung engine): keep the arena pinned
        and mapped for the life of the process (``finalize`` skips the unregistration)."""
        self._quarantined = True

    def add_finalizer(self, fn) -> None:
        """Run ``fn()`` in ``finalize`` after the shutdown signal and before the arena is
        unpinned: consumers with native threads on the arena (the stager) stop there,
        even when the loader itself was never closed (an exception unwound the job)."""
        self._finalizers.append(fn)

    def remove_finalizer(self, fn) -> None:
        try:
            self._finalizers.remove(fn)
        except ValueError:
            pass

    def finalize(self, join_timeout_s: float = 10.0) -> None:
        if self._closed:
            return
        self._closed = True
        self.shutdown_operation()
        for fn in self._finalizers:
            try:
                fn()
            except Exception as e:  # pragma: no cover - best effort
                logger.warning("finalizer %r failed: %s", fn, e)
        self._finalizers.clear()
        for proc in self.processes:
            if proc is None:
                continue
            proc.join(join_timeout_s)
            if proc.is_alive() and hasattr(proc, "terminate"):
                logger.warning("producer pid %s did not exit; terminating", proc.pid)
                proc.terminate()
                proc.join(5)
        if self._registered and self.arena is not None and not getattr(self, "_quarantined", False):
            try:
                torch.cuda.synchronize()
                _native.hip().host_unregister(self.arena.base_address)
            except Exception as e:  # pragma: no cover
                logger.warning("hipHostUnregister failed: %s", e)
            self._registered = False

    def kill(self) -> None:
        """Job abort (``parallel/abort.py``): stop the producers NOW -- no joins, no device sync (the
        GPU may be stuck behind a collective that will never complete). The arena file is already
        unlinked, so nothing is left in /dev/shm."""
        if self._closed:  # finalized already (its arena may be unmapped): nothing left to stop
            return
        self._closed = True
        if self.arena is not None:
            self.arena.request_shutdown()
        for proc in self.processes:
            if proc is not None and hasattr(proc, "kill"):
                try:
                    proc.kill()
                except Exception:  # pragma: no cover - already gone
                    pass

    def producer_stats(self) -> list[dict]:
        if self.arena is None:
            return []
        return [self.arena.producer_info(i) for i in range(self.n_producers)]


@for_all_methods(with_logging, exclude=["Istart_access_epoch", "Iend_access_epoch", "poll_control"])
class ProducerConnection:
    """Producer-side end: pipe to the consumer + the attached arena."""

    role = "producer"

    def __init__(self, pipe, producer_index: int, consumer_pid: int, timeout_s: float = DEFAULT_TIMEOUT_S):
        self.pipe = _Pipe(pipe, None, "consumer")
        self.index = producer_index
        self.consumer_pid = consumer_pid
        self.timeout_s = timeout_s
        self.arena = None

    def recv_metadata_as_producer(self) -> MetaData_Consumer_To_Producer:
        return self.pipe.recv("meta", self.timeout_s)

    def send_metadata(self, metadata: MetaData_Producer_To_Consumer, called_from: str = "producer") -> None:
        if called_from != "producer":
            raise ValueError(f"{called_from=} is not valid on the producer side")
        self.pipe.send("meta", metadata)

    def attach_windows(self, shape: tuple[int, ...], dtype: torch.dtype) -> list[tuple[Any, torch.Tensor]]:
        name = self.pipe.recv("arena", self.timeout_s)
        rt = _native.runtime()
        self.arena = rt.Arena.attach(name)
        self.arena.set_producer_pid(self.index, os.getpid())
        self.pipe.send("attached")
        return [_window_view(self.arena, self.index, s, tuple(shape), dtype) for s in range(self.arena.n_slots)]

    def Barrier(self) -> None:  # noqa: N802
        self.pipe.send("barrier")
        self.pipe.recv("barrier", self.timeout_s)

    def sync(self, target: int = 0) -> None:
        """Reference ``Win.Sync`` (ddl/connection.py:61-63): ordering comes from the
        release/acquire slot state word, see ``Connection.sync``."""

    _sync = sync

    def poll_control(self):
        """Non-blocking: a pending control message from the consumer, ``(tag, payload)`` or None.

        ``("seek", None)``: the consumer is repositioning the producers (live
        ``load_state_dict`` / ``set_epoch``); answer with :meth:`pause_for_seek`.
        """
        if not self.pipe.conn.poll(0):
            return None
        try:
            return self.pipe.conn.recv()
        except (EOFError, OSError):
            return None

    def pause_for_seek(self) -> int:
        """Acknowledge a seek and block until the consumer names the round to continue from."""
        self.pipe.send("seek_ack")
        return int(self.pipe.recv("go", self.timeout_s))

    def Istart_access_epoch(self, slot: int) -> WorkerInfo:  # noqa: N802
        """Wait until the consumer hands ``slot`` back (EMPTY), or shutdown."""
        rt = _native.runtime()
        rc = self.arena.wait_state(self.index, slot, rt.EMPTY, int(self.timeout_s * 1000), self.consumer_pid, -1)
        if rc == rt.WaitResult.OK:
            return WorkerInfo.CONTINUE
        if rc == rt.WaitResult.SHUTDOWN:
            return WorkerInfo.STOP
        _raise_for(rc, f"producer {self.index} waiting for slot {slot}", None, self.consumer_pid)
        return WorkerInfo.STOP  # pragma: no cover

    def Iend_access_epoch(self, slot: int, seq: int, used_bytes: int, epoch: int = 0,  # noqa: N802
                          tags: list[int] | None = None) -> WorkerInfo:
        """Publish ``slot`` (READY) to the consumer."""
        if self.arena.shutdown_requested():
            return WorkerInfo.STOP
        self.arena.publish(self.index, slot, seq, used_bytes, epoch, tags or [])
        return WorkerInfo.CONTINUE

    def report_error(self, exc: BaseException) -> None:
        tb = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))
        try:
            if self.arena is not None:
                self.arena.mark_failed(self.index)
        finally:
            try:
                self.pipe.send("error", tb)
            except (BrokenPipeError, OSError):
                pass

    def finalize(self) -> None:
        if self.arena is not None:
            self.arena.set_producer_status(self.index, _native.runtime().STATUS_DONE)
