"""File-backed producer read path: native coalesced pread (buffered / O_DIRECT) vs np.memmap fancy-indexing.

Writes a synthetic [N, 3, 224, 224] uint8 file, then times reading random 256-sample
batches into a pinned-size host buffer, the way an IndexedProducer fills its slot.
Prints one JSON line per variant.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ddl_amd.models import FileRowsSource  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default=os.path.join(os.path.dirname(__file__), "..", "build", "bench_rows.bin"))
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4, 8])
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    shape = (3, 224, 224)
    row = int(np.prod(shape))
    os.makedirs(os.path.dirname(a.path), exist_ok=True)
    if not os.path.exists(a.path) or os.path.getsize(a.path) != a.n * row:
        rng = np.random.default_rng(0)
        with open(a.path, "wb") as f:
            for c in range(0, a.n, 512):
                f.write(rng.integers(0, 255, size=(min(512, a.n - c), row), dtype=np.uint8).tobytes())
    rng = np.random.default_rng(1)
    batches = [rng.permutation(a.n)[: a.batch] for _ in range(a.batches)]
    out = np.empty((a.batch, row), np.uint8)
    mm = np.memmap(a.path, np.uint8, "r", shape=(a.n, row))
    t0 = time.perf_counter()
    for idx in batches:
        out[:] = mm[idx]
    dt = time.perf_counter() - t0
    print(json.dumps({"variant": "np.memmap fancy index", "threads": 1,
                      "samples_per_s": round(a.batch * a.batches / dt, 1),
                      "GBps": round(a.batch * a.batches * row / dt / 1e9, 2)}))
    for direct in (False, True):
        src = FileRowsSource(a.path, shape, "uint8", direct=direct)
        for th in a.threads:
            src.gather(batches[0], out.ctypes.data, th)  # warm the pool
            t0 = time.perf_counter()
            for idx in batches:
                src.gather(idx, out.ctypes.data, th)
            dt = time.perf_counter() - t0
            assert np.array_equal(out, mm[batches[-1]])
            print(json.dumps({"variant": "native pread" + (" O_DIRECT" if direct else " buffered"),
                              "threads": th, "has_direct": src._file().has_direct,
                              "samples_per_s": round(a.batch * a.batches / dt, 1),
                              "GBps": round(a.batch * a.batches * row / dt / 1e9, 2)}))
        src.close()
    if not a.keep:
        os.unlink(a.path)


if __name__ == "__main__":
    main()
