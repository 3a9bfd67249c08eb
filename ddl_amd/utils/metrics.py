"""JSON-lines metrics emitter (SURVEY §5 "Metrics / logging / observability").

``MetricsWriter(loader, path)`` appends one JSON record per ``interval_s`` (or
per ``flush()``) with the loader's counters: samples, batches, samples/s since
the previous record, bytes staged H2D, consumer wait time, producer fill/wait
times from the native heartbeat records, and (when given a
``ComputeIdleMeter``) the compute stream's idle %. Rank-tagged; cheap (no
device sync unless an idle meter is attached).
"""

from __future__ import annotations

import json
import os
import time
from typing import Any


class MetricsWriter:
    def __init__(self, loader: Any, path: str, interval_s: float = 10.0, idle_meter: Any = None):
        self.loader = loader
        self.path = path
        self.interval_s = interval_s
        self.idle_meter = idle_meter
        self._last_t = time.perf_counter()
        self._last_samples = 0
        self.rank = int(os.environ.get("RANK", "0") or 0)
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)

    def _record(self) -> dict:
        st = self.loader.stats() if hasattr(self.loader, "stats") else {}
        now = time.perf_counter()
        samples = int(st.get("samples", st.get("batches", 0)))
        rate = (samples - self._last_samples) / max(now - self._last_t, 1e-9)
        self._last_t, self._last_samples = now, samples
        rec = {"ts": time.time(), "rank": self.rank, "samples_per_s": round(rate, 2)}
        for k, v in st.items():
            if k == "producers":
                rec["producer_fill_s"] = [round(p["fill_ns_total"] / 1e9, 4) for p in v]
                rec["producer_wait_s"] = [round(p["wait_ns_total"] / 1e9, 4) for p in v]
                rec["producer_rounds"] = [p["rounds"] for p in v]
            elif isinstance(v, (int, float, str)) or v is None:
                rec[k] = v
        if self.idle_meter is not None:
            rec.update(self.idle_meter.result())
        return rec

    def step(self) -> None:
        if time.perf_counter() - self._last_t >= self.interval_s:
            self.flush()

    def flush(self) -> dict:
        rec = self._record()
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
        return rec
