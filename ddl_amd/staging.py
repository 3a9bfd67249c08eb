"""Device staging engine: producer windows -> HBM on a dedicated prefetch stream.

The reference never moves data to a GPU (``.to(device)`` is commented out at
reference tests/run_ddl.py:233-235; pinned memory / H2D is a TODO at
ddl/connection.py:89-92). This is the MI355X-native replacement of that gap
(SURVEY §2.3 ``csrc/staging``, §7.2 step 4):

* a native C++ stager thread (``csrc/kernels/stager.cpp``, no GIL) walks the
  consumer's window schedule ahead of the training loop: it futex-waits for
  producer ``p`` to publish slot ``s`` and copies it from the pinned arena into
  HBM ring buffer ``w % n_buffers`` straight on an SDMA engine through ROCr
  (direct DMA; two engines alternate). A second native thread retires the copies
  in order and hands each slot back to its producer the moment its DMA lands --
  the consumer thread is never involved. Without direct DMA (ROCr refuses: see
  ``direct_dma_reason``) the copies run on two HIP copy streams instead;
* optional post-copy device work (the cross-GPU global shuffle exchange over
  RCCL, ``parallel/shuffle.py``) on a second stream. Collectives must be
  issued in the same order and number on every rank, so they are NOT issued
  by the stager (whose progress depends on producer timing): the consumer
  thread issues window w+1's exchange when it starts window w (``get``),
  i.e. one window ahead, deterministically -- after a host wait for w+1's copy
  (no HIP event follows a direct-DMA copy);
* consumers wait for a copy on the host (``wait_ready``: a bounded wait on its
  completion signal), so no AQL queue holds a packet waiting on a copy; with a
  post-copy stage the compute stream waits on the stage's ``ready`` event;
* a buffer is recycled only after a ``free`` event recorded on the compute
  stream when the consumer moved past the window, so in-flight kernels that
  read it (permute/cast/collate) finish first.

Every host wait is bounded by the loader's ``timeout_s``: a copy that never lands raises
``DDLTimeoutError`` naming the window and SDMA engine, and ``close()`` never hangs on one.

HBM is plentiful on MI355X (288 GB): windows are staged whole, ``depth``
windows deep (default 4), plus
two ring buffers for the exchange lookahead when the exchange is on.
"""

from __future__ import annotations

import dataclasses
import sys
import time
from typing import Callable

import torch

from . import _native
from .exceptions import DDLError, DDLTimeoutError, NativeExtensionError, PeerDeathError, ShutdownError
from .utils import streams
from .utils.logging import logger
from .utils.tracing import trace_range

# window copies go straight to SDMA engines through ROCr (NativeStager direct-DMA mode) instead of HIP copy
# streams, so no AQL queue holds a packet waiting on a copy: GPU idle at r = 0.9 1.25% -> 0.78%, feed-bound
# rate 187.9k -> 191.4k samples/s (archive/profiles/r4_twentieth). With a post-copy stage (the exchange) the
# consumer waits for the copy on the host before it enqueues the stage. False: HIP copy streams (tests compare
# the two paths).
DIRECT_DMA = True


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
    meta: tuple = ()  # the window's first meta_bytes as int64 (multi-batch windows' per-batch metadata)


_SDMA_WARM: set = set()
# (ring buffers, arena, native stager) of stagers closed with copies still pending on a stuck engine: never freed
_QUARANTINE: list = []


def warm_copy_engines(device: torch.device, n_engines: int = 4, nbytes: int = 512 << 20) -> float:
    """Bring up the SDMA copy engines this process's H2D copies will use, once per device.

    The HIP runtime spreads back-to-back async copies over the GPU's SDMA engines: each copy goes to
    the lowest-numbered engine that is idle at enqueue time. The FIRST copy an engine runs in a
    process costs the enqueueing thread 6.5-11 ms (engine bring-up, measured with AMD_LOG_LEVEL=4:
    ``archive/profiles/r2_sdma_warmup``). The stager enqueues copies while earlier ones are still in
    flight, so its 2nd and 3rd engines came up in the middle of a run -- a 6.5 ms stall of the
    stager thread each time, i.e. a hole of ~5 windows of H2D in a short benchmark.
    Here ``n_engines`` copies of ``nbytes`` are enqueued on separate streams back to back, each
    long enough to keep its engine busy while the next one comes up. Returns the seconds spent.
    """
    key = (device.type, device.index)
    if key in _SDMA_WARM or device.type != "cuda":
        return 0.0
    _SDMA_WARM.add(key)
    t0 = time.perf_counter()
    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dsts = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(n_engines)]
    ss = [torch.cuda.Stream(device=device) for _ in range(n_engines)]
    for d, st in zip(dsts, ss):
        with streams.on_stream(st):
            d.copy_(src, non_blocking=True)
    for st in ss:
        st.synchronize()
    del src, dsts
    return time.perf_counter() - t0


class WindowStager:
    """Python face of the native stager (``_ddl_hip.NativeStager``).

    Window ``w`` comes from producer ``w % P``, slot ``(w // P) % n_slots`` (the
    consumer's round-robin schedule).
    """

    def __init__(self, connection, n_slots: int, total_windows: int, depth: int, device: torch.device,
                 max_window_bytes: int, post_copy: Callable | None = None, timeout_s: float = 600.0,
                 first_window: int = 0, meta_bytes: int = 0, copy_timing: bool = False):
        if depth < 1:
            raise ValueError("prefetch depth must be >= 1")
        hip, rt = _native.hip(), _native.runtime()
        self.sdma_warm_s = warm_copy_engines(torch.device(device))
        if hip.ARENA_ABI != rt.ARENA_ABI:
            raise NativeExtensionError("_ddl_hip and _ddl_runtime disagree on the Arena layout: rebuild both")
        self.conn = connection
        self.total = total_windows
        self.depth = depth
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.post_copy = post_copy
        self.timeout_s = timeout_s
        self.first = first_window
        # H2D copies run on the copy stream; post-copy device work (the RCCL
        # exchange) on a second stream, so window w's exchange overlaps window
        # w+1's DMA instead of idling the copy engine.
        self.copy_stream = torch.cuda.Stream(device=self.device)
        # two copy streams / SDMA engines, strictly alternating: when copies run back to back the next one is
        # already running when one finishes, so the ~25 us gap per copy on one engine is gone (+1.8-2.5%,
        # archive/profiles/r2_copy_streams)
        self.copy_stream2 = torch.cuda.Stream(device=self.device)
        self.stream = torch.cuda.Stream(device=self.device) if post_copy is not None else self.copy_stream
        # The consumer posts window w+1's exchange when it enters window w (the fixed, rank-identical
        # issue point of the collective, parallel/order.py), so two windows are held at once (w being
        # consumed, w+1 exchanged ahead): one extra ring buffer, and `depth` windows of DMA behind them.
        n_buf = depth + 1 if post_copy is not None else depth
        self.max_window_bytes = int(max_window_bytes)
        self.buffers = [torch.empty(max_window_bytes, dtype=torch.uint8, device=self.device) for _ in range(n_buf)]
        self.ready_events = [torch.cuda.Event() for _ in range(n_buf)]
        self._copy_done = [torch.cuda.Event() for _ in range(n_buf)]
        for ev in self.ready_events + self._copy_done:  # materialise the hipEvents (lazy in torch)
            ev.record(self.copy_stream)
        self._free_refs: list[list] = [[] for _ in range(n_buf)]  # keep free events alive for the stager
        self._staged: dict[int, StagedWindow] = {}
        self._posted: set[int] = set()
        self._closed = False
        self._n_released = 0
        self.post_wait_s = 0.0  # host time blocked at a collective issue point waiting for its window
        self.post_waits: list[float] = []  # ... per posted window (seconds), for the p50 / p99 in stats()
        self._native = hip.NativeStager(
            arena=connection.arena.address, n_producers=connection.n_producers, n_slots=n_slots,
            first=first_window, total=total_windows, buffers=[b.data_ptr() for b in self.buffers],
            buffer_bytes=max_window_bytes, copy_stream=self.copy_stream.cuda_stream, device=self.device.index,
            peer_pids=list(connection.producer_pids), timeout_ms=int(timeout_s * 1000),
            ready=[e.cuda_event for e in self.ready_events], copy_done=[e.cuda_event for e in self._copy_done],
            post_copy=post_copy is not None, meta_bytes=int(meta_bytes),
            copy_stream2=self.copy_stream2.cuda_stream, direct_dma=bool(DIRECT_DMA), copy_timing=bool(copy_timing))
        self.direct_dma = bool(self._native.direct_dma)
        if DIRECT_DMA and not self.direct_dma:
            logger.info("direct-DMA staging unavailable (%s): HIP copy streams", self._native.direct_dma_reason)
        # the stream fallback too waits for a pending free ring buffer on the host (polled, close() interrupts
        # it) instead of a barrier packet in the copy stream's queue: GPU idle near r = 1 1.4-1.6% -> 0.9-1.0%
        # (archive/profiles/r4_seventeenth)
        self._native.free_on_host = True
        self.copy_streams = 2
        self.meta_bytes = int(meta_bytes)

    # -------------------------------------------------------------- consumer
    def _wrap(self, info: dict) -> StagedWindow:
        w = int(info["window"])
        sw = self._staged.get(w)
        if sw is None:
            b, n = int(info["buffer"]), int(info["used_bytes"])
            sw = StagedWindow(w, b, int(info["producer"]), int(info["slot"]), int(info["seq"]), n,
                              self.buffers[b][:n], float(info["t_ready_host"]), tuple(info["tag"]),
                              tuple(info["meta"]))
            self._staged[w] = sw
        return sw

    def get(self, w: int) -> StagedWindow:
        """Window ``w`` staged in HBM; the current stream is made to wait for it (device-side)."""
        if self.post_copy is not None:
            self._post(w)  # normally already posted by post() at the previous window's hand-back
        sw = self._wait_staged(w)
        self.wait_ready(sw, streams.current(self.device.index))
        return sw

    def wait_ready(self, sw: StagedWindow, stream) -> None:
        """Order ``stream`` after window ``sw``'s copy (and its post-copy stage): a device-side event wait, or in
        direct-DMA mode without a post-copy stage (no HIP event behind the copy) a host wait for the copy's
        completion signal, bounded by ``timeout_s``."""
        if self.direct_dma and self.post_copy is None:
            self._wait_copy(sw.index)
        else:
            stream.wait_event(self.ready_events[sw.buffer])

    def _wait_copy(self, w: int) -> None:
        """Host wait for window ``w``'s H2D copy (the stager's bounded wait; GIL released)."""
        rc = self._native.wait_copy(w)
        if rc == 0:
            return
        if rc == 2:
            raise DDLTimeoutError(self._native.error() or f"window {w}: its H2D copy did not land within "
                                                          f"{self.timeout_s:.0f}s")
        if rc == 1:
            raise ShutdownError(f"window {w}: loader was shut down while waiting for its copy")
        raise DDLError(f"window {w}: waiting for its copy failed ({self._native.error()})")

    def peek(self, w: int) -> StagedWindow | None:
        """Window ``w`` if it is already staged AND its post-copy work (exchange) is
        issued, else None -- never blocks, never issues collectives."""
        if self.post_copy is not None and w not in self._posted:
            return None
        sw = self._staged.get(w)
        if sw is not None:
            return sw
        info = self._native.peek(w)
        return None if info is None else self._wrap(info)

    def post(self, w: int) -> None:
        """Issue window ``w``'s post-copy work (the exchange collective) now, from the consumer
        thread; waits on the host until ``w`` is staged. A no-op without post-copy work."""
        if self.post_copy is not None and w < self.first + self.total:
            self._post(w)

    def _post(self, w: int) -> None:
        if w in self._posted:
            return
        t0 = time.perf_counter()
        sw = self._wait_staged(w)
        if self.direct_dma:  # no HIP event behind the copy: the host waits for it, then enqueues the stage
            self._wait_copy(w)
        else:
            self.stream.wait_event(self._copy_done[sw.buffer])
        dt = time.perf_counter() - t0  # the issue point's host wait: producer publish + (direct DMA) the copy
        self.post_wait_s += dt
        self.post_waits.append(dt)
        with streams.on_stream(self.stream), trace_range("ddl.stage.post_copy"):
            self.post_copy(sw.data, w, {"seq": sw.seq, "used_bytes": sw.nbytes, "tag": list(sw.tags)})
        self.ready_events[sw.buffer].record(self.stream)
        self._posted.add(w)

    def _wait_staged(self, w: int) -> StagedWindow:
        sw = self._staged.get(w)
        if sw is not None:
            return sw
        if self._closed:
            raise ShutdownError("stager stopped")
        with trace_range("ddl.stage.wait"):
            rc, producer, info = self._native.wait(w, int(self.timeout_s * 1000))
        if rc == 0:
            return self._wrap(info)
        what = f"staging window {w}"
        if rc == -1:
            raise DDLError(f"{what}: {self._native.error()}")
        if rc == 2:
            raise DDLTimeoutError(f"{what}: not staged within {self.timeout_s:.0f}s (producer {producer})")
        if rc == 1:
            raise ShutdownError(f"{what}: loader was shut down")
        pids = self.conn.producer_pids
        pid = pids[producer] if 0 <= producer < len(pids) else None
        if rc == 4:
            raise PeerDeathError(f"{what}: producer {producer} reported a failure", producer, pid)
        raise PeerDeathError(f"{what}: producer {producer} (pid {pid}) died", producer, pid)

    def forget(self, w: int) -> None:
        """Drop the Python-side record of window ``w`` (the native batch engine handed its buffer back)."""
        self._staged.pop(w, None)
        self._posted.discard(w)

    def release(self, w: int, stream: torch.cuda.Stream | None = None, event: torch.cuda.Event | None = None) -> None:
        """Consumer is done with window ``w`` as of ``stream``'s position (default: the current
        stream): every kernel that reads the window must be on that stream, before this call.
        ``event``: an already-recorded event after the last read of the window (used as is)."""
        sw = self._staged.pop(w, None)
        if sw is None:
            return
        self._posted.discard(w)
        self._n_released += 1
        if event is not None:
            ev = event
        else:
            ev = torch.cuda.Event()
            ev.record(stream if stream is not None else streams.current(self.device.index))
        refs = self._free_refs[sw.buffer]
        refs.append(ev)
        del refs[:-2]  # the stager has enqueued its wait on the older one by now
        self._native.release(w, ev.cuda_event)

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        self._native.close()
        if self._native.poisoned:
            # a copy never landed and copies were still queued behind it: an engine may write the ring (and
            # read the arena) at any later time, so neither is freed -- nor are the copy streams waited for
            self._quarantine()
            return
        self.copy_stream.synchronize()
        self.copy_stream2.synchronize()
        self.stream.synchronize()
        # drop the ring (a live seek builds a new stager; batches handed out keep their own refs) and any
        # token-collate views cached over it (models/tokens.py), which would otherwise keep it allocated
        self._staged.clear()
        tok = sys.modules.get("ddl_amd.models.tokens")
        if tok is not None:
            tok.drop_cached_views(b.data_ptr() for b in self.buffers)
        self.buffers = []

    def _quarantine(self) -> None:
        """Keep the HBM ring and the pinned arena alive for the life of the process (module-level refs; the
        connection skips the arena's hipHostUnregister) -- the price of a hung copy engine is a leak, never a
        late DMA write into freed or reused memory."""
        _QUARANTINE.append((self.buffers, self.conn.arena, self._native))
        quarantine = getattr(self.conn, "quarantine", None)
        if quarantine is not None:
            quarantine()
        logger.warning("stager closed with copies pending on a stuck engine: %d ring buffers (%.1f MB) and the "
                       "arena stay allocated; %d completion signals leaked", len(self.buffers),
                       len(self.buffers) * self.max_window_bytes / 1e6, int(self._native.leaked_signals))
        self._staged.clear()
        self.buffers = []

    @property
    def poisoned(self) -> bool:
        """A copy wait failed with copies pending (see ``_quarantine``)."""
        return bool(self._native.poisoned)

    @property
    def bytes_h2d(self) -> int:
        return int(self._native.bytes_h2d)

    @property
    def windows_staged(self) -> int:
        """Windows whose H2D copy has been enqueued."""
        return int(self._native.windows_staged)

    def settle(self, timeout_s: float = 1.0) -> None:
        """After a device synchronize: wait until every completed copy has been counted as landed."""
        self._native.settle(int(timeout_s * 1000))

    @property
    def copy_timing(self) -> bool:
        """Device times for every window copy, which ``bytes_in_interval`` / ``copy_summary`` need. Direct DMA
        takes them from ROCr's async-copy profiling, a PROCESS-WIDE switch (it timestamps every async copy of
        the process, torch's and RCCL's included), so it is off unless set here; turn it on before the copies
        to be measured. Stream-mode copies are always timed."""
        return bool(self._native.copy_timing)

    @copy_timing.setter
    def copy_timing(self, on: bool) -> None:
        if not self._native.set_copy_timing(bool(on)):
            raise DDLError("ROCr refused async-copy profiling: no device times for direct-DMA copies")

    def bytes_in_interval(self, e0: torch.cuda.Event, e1: torch.cuda.Event, timeout_s: float = 2.0) -> dict:
        """H2D bytes that crossed PCIe between two recorded timing events (``enable_timing=True``), on the
        GPU clock: each copy is timed on the device and counts with the share of its bytes whose [start, end]
        lies between the events. ``{"ok", "bytes", "windows", "copies", "t0_ms", "t1_ms", "untimed",
        "truncated"}``; waits (bounded) for copies still in flight. ``ok`` is False when a copy that may
        overlap the interval was not timed (``copy_timing`` off when it ran) or its record was dropped."""
        return dict(self._native.bytes_in_interval(e0.cuda_event, e1.cuda_event, int(timeout_s * 1000)))

    def copy_summary(self, e0: torch.cuda.Event, e1: torch.cuda.Event) -> dict:
        """How the window copies ran between two timing events: copies per stream, link busy % and the share
        with two copies in flight."""
        pro = self.bytes_in_interval(e0, e1)
        span = max(1e-9, pro.get("t1_ms", 0.0) - pro.get("t0_ms", 0.0))
        out: dict = {}
        if pro.get("ok"):
            out.update(copies_per_stream=list(pro["copies_per_stream"]),
                       link_busy_pct=round(100.0 * pro["busy_ms"] / span, 2),
                       two_copies_pct=round(100.0 * pro["overlap_ms"] / span, 2))
        return out

    @property
    def windows_landed(self) -> int:
        """Windows whose H2D copy has retired (the data is in HBM)."""
        return int(self._native.windows_landed)

    @property
    def bytes_landed(self) -> int:
        return int(self._native.bytes_landed)

    @property
    def windows_released(self) -> int:
        """Windows the consumer has handed back (fully consumed)."""
        return self._n_released

    def stats(self) -> dict:
        return {"bytes_h2d": self.bytes_h2d, "windows_staged": self.windows_staged,
                "windows_landed": self.windows_landed, "bytes_landed": self.bytes_landed,
                "stager_wait_producer_s": float(self._native.wait_producer_s),
                "copy_streams": self.copy_streams, "free_waits_enqueued": int(self._native.free_waits),
                "free_on_host": bool(self._native.free_on_host), "direct_dma": self.direct_dma,
                "direct_dma_reason": self._native.direct_dma_reason,
                "exchange_issue_wait_s": round(self.post_wait_s, 6),
                **issue_wait_summary(self.post_waits)}


def issue_wait_summary(waits: list[float]) -> dict:
    """p50 / p99 / max (ms) of the per-window host waits at the exchange's issue point (empty without one)."""
    if not waits:
        return {}
    s = sorted(waits)

    def q(p: float) -> float:
        return round(1e3 * s[min(len(s) - 1, int(p * (len(s) - 1) + 0.5))], 4)

    return {"exchange_issue_wait_n": len(s), "exchange_issue_wait_p50_ms": q(0.50),
            "exchange_issue_wait_p99_ms": q(0.99), "exchange_issue_wait_max_ms": round(1e3 * s[-1], 4)}
