"""Device staging engine: producer windows -> HBM on a dedicated prefetch stream.

The reference never moves data to a GPU (``.to(device)`` is commented out at
reference tests/run_ddl.py:233-235; pinned memory / H2D is a TODO at
ddl/connection.py:89-92). This is the MI355X-native replacement of that gap
(SURVEY §2.3 ``csrc/staging``, §7.2 step 4):

* a background *staging thread* walks the consumer's window schedule ahead of
  the training loop: it waits (GIL released, futex) for producer ``p`` to
  publish slot ``s``, enqueues ``hipMemcpyAsync`` H2D from the pinned arena
  into HBM buffer ``w % depth`` on the **prefetch stream**, then enqueues
  (``hipLaunchHostFunc``) the hand-back of the slot to its producer, so the
  producer refills it the moment the DMA retires -- the consumer thread is
  never involved;
* optional post-copy device work (the cross-GPU global shuffle exchange over
  RCCL, ``parallel/shuffle.py``) on a second stream. Collectives must be
  issued in the same order and number on every rank, so they are NOT issued
  by the staging thread (whose progress depends on producer timing): the
  consumer thread issues window w+1's exchange when it starts window w
  (``get``), i.e. one window ahead, deterministically;
* a ``ready`` event per buffer; the compute stream waits on it *on the device*
  (``hipStreamWaitEvent``) -- the host never blocks on a copy;
* a buffer is recycled only after a ``free`` event recorded on the compute
  stream when the consumer moved past the window, so in-flight kernels that
  read it (permute/cast/collate) finish first.

HBM is plentiful on MI355X (288 GB): windows are staged whole, ``depth``
windows deep (default 2 = double buffering against the training step).
"""

from __future__ import annotations

import dataclasses
import threading
import time
from typing import Callable

import torch

from . import _native
from .exceptions import DDLTimeoutError, ShutdownError
from .utils.logging import logger
from .utils import streams
from .utils.tracing import trace_range


@dataclasses.dataclass
class StagedWindow:
    index: int
    buffer: int
    producer: int
    slot: int
    seq: int
    nbytes: int
    data: torch.Tensor  # uint8 view [nbytes] of the HBM buffer
    t_ready_host: float
    tags: tuple = ()


class WindowStager:
    def __init__(self, connection, schedule: Callable[[int], tuple[int, int]], total_windows: int, depth: int,
                 device: torch.device, max_window_bytes: int, post_copy: Callable | None = None,
                 timeout_s: float = 600.0, first_window: int = 0):
        if depth < 1:
            raise ValueError("prefetch depth must be >= 1")
        self.conn = connection
        self.schedule = schedule
        self.total = total_windows
        self.depth = depth
        self.device = torch.device(device)
        self.post_copy = post_copy
        self.timeout_s = timeout_s
        self.first = first_window
        # H2D copies run on the copy stream; post-copy device work (the RCCL
        # exchange) on a second stream, so window w's exchange overlaps window
        # w+1's DMA instead of idling the copy engine.
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.stream = torch.cuda.Stream(device=self.device) if post_copy is not None else self.copy_stream
        self._copy_done = [torch.cuda.Event() for _ in range(depth)]
        self.buffers = [torch.empty(max_window_bytes, dtype=torch.uint8, device=self.device) for _ in range(depth)]
        self.ready_events = [torch.cuda.Event() for _ in range(depth)]
        self.free_events: list[torch.cuda.Event | None] = [None] * depth
        self._cv = threading.Condition()
        self._staged: dict[int, StagedWindow] = {}
        self._infos: dict[int, dict] = {}
        self._posted: set[int] = set()
        self._released_upto = first_window  # windows < this are released by the consumer
        self._stop = False
        self._error: BaseException | None = None
        self.bytes_h2d = 0
        self.windows_staged = 0
        self.wait_producer_s = 0.0
        self._hip = _native.hip()
        self._thread = threading.Thread(target=self._run, name="ddl-stager", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------ background
    def _run(self) -> None:
        try:
            torch.cuda.set_device(self.device)
            handle = self.copy_stream.cuda_stream
            for w in range(self.first, self.first + self.total):
                b = (w - self.first) % self.depth
                with self._cv:
                    while not self._stop and w - self.depth >= self._released_upto:
                        self._cv.wait(0.1)
                    if self._stop:
                        return
                    free_ev = self.free_events[b]
                if free_ev is not None:
                    self.copy_stream.wait_event(free_ev)
                p, s = self.schedule(w)
                t0 = time.perf_counter()
                with trace_range("ddl.stage.wait_producer"):
                    info = self.conn.acquire(p, s, self.timeout_s)
                self.wait_producer_s += time.perf_counter() - t0
                nbytes = int(info["used_bytes"])
                buf = self.buffers[b]
                if nbytes > buf.numel():
                    raise RuntimeError(f"window of {nbytes} B exceeds staging buffer of {buf.numel()} B")
                with trace_range("ddl.stage.h2d"):
                    self._hip.memcpy_h2d(buf.data_ptr(), self.conn.slot_address(p, s), nbytes, handle)
                self.conn.release_on_stream(p, s, handle)
                view = buf[:nbytes]
                if self.post_copy is not None:
                    self._copy_done[b].record(self.copy_stream)  # post_copy runs later, from get()
                else:
                    self.ready_events[b].record(self.copy_stream)
                self.bytes_h2d += nbytes
                self.windows_staged += 1
                with self._cv:
                    self._staged[w] = StagedWindow(w, b, p, s, int(info["seq"]), nbytes, view, time.perf_counter(),
                                                   tuple(info["tag"]))
                    self._infos[w] = info
                    self._cv.notify_all()
        except ShutdownError:
            pass
        except BaseException as e:  # surfaced to the consumer on its next get()
            logger.error("staging thread failed: %r", e)
            with self._cv:
                self._error = e
                self._cv.notify_all()

    # -------------------------------------------------------------- consumer
    def get(self, w: int) -> StagedWindow:
        """Window ``w`` staged in HBM; the current stream is made to wait for it (device-side)."""
        if self.post_copy is not None:
            self._post(w)
            if self.depth >= 2 and w + 1 < self.first + self.total:
                self._post(w + 1)  # one window ahead, in lockstep on every rank
        sw = self._wait_staged(w)
        streams.current(self.device.index).wait_event(self.ready_events[sw.buffer])
        return sw

    def peek(self, w: int) -> StagedWindow | None:
        """Window ``w`` if it is already staged AND its post-copy work (exchange) is
        issued, else None -- never blocks, never issues collectives."""
        with self._cv:
            sw = self._staged.get(w)
        if sw is None or (self.post_copy is not None and w not in self._posted):
            return None
        return sw

    def _post(self, w: int) -> None:
        if w in self._posted:
            return
        sw = self._wait_staged(w)
        with self._cv:
            info = self._infos.pop(w, {})
        self.stream.wait_event(self._copy_done[sw.buffer])
        with torch.cuda.stream(self.stream), trace_range("ddl.stage.post_copy"):
            self.post_copy(sw.data, w, info)
        self.ready_events[sw.buffer].record(self.stream)
        self._posted.add(w)

    def _wait_staged(self, w: int) -> StagedWindow:
        deadline = time.monotonic() + self.timeout_s
        with self._cv:
            while w not in self._staged:
                if self._error is not None:
                    raise self._error
                if self._stop:
                    raise ShutdownError("stager stopped")
                if time.monotonic() > deadline:
                    raise DDLTimeoutError(f"window {w} was not staged within {self.timeout_s:.0f}s")
                self._cv.wait(0.05)
            return self._staged[w]

    def release(self, w: int) -> None:
        """Consumer is done with window ``w`` (as of the current stream position)."""
        with self._cv:
            sw = self._staged.pop(w, None)
            if sw is None:
                return
            self._posted.discard(w)
            ev = torch.cuda.Event()
            ev.record(streams.current(self.device.index))
            self.free_events[sw.buffer] = ev
            self._released_upto = max(self._released_upto, w + 1)
            self._cv.notify_all()

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(timeout=30)
        if self._thread.is_alive():  # pragma: no cover
            logger.warning("staging thread did not exit")
        self.copy_stream.synchronize()
        self.stream.synchronize()

    def stats(self) -> dict:
        return {"bytes_h2d": self.bytes_h2d, "windows_staged": self.windows_staged,
                "stager_wait_producer_s": self.wait_producer_s}
