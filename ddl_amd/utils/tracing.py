"""Tracing and metrics (the reference has DEBUG logs only).

* ``trace_range(name)``: roctx range (via torch's ROCm ``nvtx`` shim, which is
  backed by libroctx64) around produce / stage / consume phases, visible in
  ``rocprofv3 --marker-trace``; a no-op when unavailable or disabled
  (``DDL_ROCTX=0``).
* ``LoaderMetrics``: host counters (samples, bytes staged H2D, consumer waits,
  producer fill/wait times).
* ``ComputeIdleMeter``: GPU idle % of the compute stream measured with HIP
  events: idle = 1 - sum(step busy) / (last step end - first step start),
  where each step's start event is recorded *after* the stream waits on the
  batch-ready event, so time spent waiting for data counts as idle.
"""

from __future__ import annotations

import dataclasses
import os
import time
from typing import Any

_ROCTX_ENABLED = os.environ.get("DDL_ROCTX", "1") != "0"


_ROCTX = None  # (push, pop) once resolved; () when markers are off or there is no GPU


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = ()
        if _ROCTX_ENABLED:
            try:
                import torch

                if torch.cuda.is_available():
                    _ROCTX = (torch.cuda.nvtx.range_push, torch.cuda.nvtx.range_pop)
            except Exception:
                _ROCTX = ()
    return _ROCTX


class trace_range:  # noqa: N801  (used like a function: ``with trace_range("name"):``)
    """roctx range around a block (a plain class: this sits on the per-batch host path)."""

    __slots__ = ("name", "pushed")

    def __init__(self, name: str):
        self.name = name
        self.pushed = False

    def __enter__(self):
        r = _ROCTX if _ROCTX is not None else _roctx()
        if r:
            r[0](self.name)
            self.pushed = True
        return self

    def __exit__(self, *exc):
        if self.pushed:
            _ROCTX[1]()
        return False


@dataclasses.dataclass
class LoaderMetrics:
    batches: int = 0
    samples: int = 0
    bytes_h2d: int = 0
    windows: int = 0
    consumer_wait_s: float = 0.0  # host time blocked waiting for a producer window
    stage_enqueue_s: float = 0.0
    t_first: float | None = None
    t_last: float | None = None

    def on_batch(self, n_samples: int) -> None:
        now = time.perf_counter()
        if self.t_first is None:
            self.t_first = now
        self.t_last = now
        self.batches += 1
        self.samples += n_samples

    def as_dict(self) -> dict[str, Any]:
        d = dataclasses.asdict(self)
        if self.t_first is not None and self.t_last is not None and self.t_last > self.t_first:
            d["samples_per_s_host"] = self.samples / (self.t_last - self.t_first)
        return d


class ComputeIdleMeter:
    """Measure the compute stream's idle fraction over a run of steps."""

    def __init__(self, stream: Any | None = None, max_steps: int = 1 << 16):
        import torch

        self._torch = torch
        self.stream = stream
        self.max_steps = max_steps
        self._pairs: list[tuple[Any, Any]] = []
        self._cur: Any | None = None

    def step_begin(self) -> None:
        if len(self._pairs) >= self.max_steps:
            return
        ev = self._torch.cuda.Event(enable_timing=True)
        ev.record(self.stream) if self.stream is not None else ev.record()
        self._cur = ev

    def step_end(self) -> None:
        if self._cur is None:
            return
        ev = self._torch.cuda.Event(enable_timing=True)
        ev.record(self.stream) if self.stream is not None else ev.record()
        self._pairs.append((self._cur, ev))
        self._cur = None

    def reset(self) -> None:
        self._pairs.clear()
        self._cur = None

    def result(self) -> dict[str, float]:
        if not self._pairs:
            return {"gpu_idle_pct": float("nan"), "busy_ms": 0.0, "wall_ms": 0.0, "steps": 0}
        self._pairs[-1][1].synchronize()
        busy = sum(s.elapsed_time(e) for s, e in self._pairs)
        wall = self._pairs[0][0].elapsed_time(self._pairs[-1][1])
        idle = 0.0 if wall <= 0 else max(0.0, 1.0 - busy / wall)
        out = {"gpu_idle_pct": 100.0 * idle, "busy_ms": busy, "wall_ms": wall, "steps": len(self._pairs)}
        if len(self._pairs) > 1:
            # where the idle sits: many small gaps at every step boundary (device-side overhead) or a few
            # long stalls (the feed running dry)
            gaps = sorted(max(0.0, 1000.0 * a[1].elapsed_time(b[0])) for a, b in zip(self._pairs, self._pairs[1:]))
            tot = sum(gaps)
            top = gaps[-max(1, len(gaps) // 100):]

            def pct(q: float) -> float:
                return round(gaps[min(len(gaps) - 1, int(q * len(gaps)))], 1)

            out["gaps_us"] = {"p50": pct(0.5), "p90": pct(0.9), "p99": pct(0.99), "max": round(gaps[-1], 1),
                              "top1pct_share": round(sum(top) / tot, 3) if tot > 0 else 0.0}
        return out
