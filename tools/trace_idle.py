#!/usr/bin/env python3
"""GPU idle % from a rocprofv3 trace: the cross-check of ``ComputeIdleMeter``.

``bench.py`` brackets its timed regions with roctx ranges ``bench.phase1`` /
``bench.phase2``. Run it under

    rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv \
        -d gpurun_out/trace -o bench -- python3 bench.py ...

and this tool reads the CSVs, clips every kernel dispatch and every copy to a
marked region and reports:

* ``device_idle_pct``: 1 - |union of all kernel intervals| / region wall time
  -- the time the GPU had no kernel at all resident (host launch gaps of the
  training step included, so it is >= the event-based number, which only
  counts the gaps *between* steps);
* ``loader_kernel_pct``: the union of the loader's own kernels (gather, cast,
  collate, checksum, exchange pack/unpack) over the wall time;
* ``copy_busy_pct``: the union of H2D copies over the wall time (the PCIe feed);
* the longest gaps with no kernel resident.

Timestamps of host markers and GPU dispatches share rocprofv3's clock (ns).
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

LOADER_KERNELS = ("move_rows", "convert_rows", "convert_u8", "checksum", "hwc", "gather", "scatter", "pad_pack",
                  "feistel", "split_columns", "pack_columns", "random_resized", "column_stats", "norm_affine")


def _rows(path: str) -> list[dict]:
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _find(d: str, suffix: str) -> list[str]:
    return sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))


def _ts(r: dict) -> tuple[int, int]:
    return int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def union_ns(intervals: list[tuple[int, int]], lo: int, hi: int) -> tuple[int, list[tuple[int, int]]]:
    """Length of the union of ``intervals`` clipped to [lo, hi], and the gaps between the merged spans."""
    clipped = sorted((max(a, lo), min(b, hi)) for a, b in intervals if b > lo and a < hi)
    total, gaps, cur_a, cur_b = 0, [], None, None
    prev_end = lo
    for a, b in clipped:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                total += cur_b - cur_a
                prev_end = cur_b
            if a > prev_end:
                gaps.append((prev_end, a))
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        total += cur_b - cur_a
        prev_end = cur_b
    if hi > prev_end:
        gaps.append((prev_end, hi))
    return total, gaps


def regions(markers: list[dict], names: tuple[str, ...]) -> dict[str, tuple[int, int]]:
    out = {}
    for r in markers:
        text = " ".join(str(v) for v in r.values())
        for n in names:
            if n in text and "Start_Timestamp" in r:
                a, b = _ts(r)
                if b > a and (n not in out or b - a > out[n][1] - out[n][0]):
                    out[n] = (a, b)
    return out


def analyse(kernels: list[dict], copies: list[dict], markers: list[dict],
            names: tuple[str, ...] = ("bench.phase1", "bench.phase2")) -> dict:
    ks = [(_ts(r), r.get("Kernel_Name", "")) for r in kernels]
    cs = [_ts(r) for r in copies]
    res = {}
    for name, (lo, hi) in sorted(regions(markers, names).items()):
        wall = hi - lo
        busy, gaps = union_ns([t for t, _ in ks], lo, hi)
        lbusy, _ = union_ns([t for t, n in ks if any(k in n for k in LOADER_KERNELS)], lo, hi)
        cbusy, _ = union_ns(cs, lo, hi)
        n_disp = sum(1 for (a, b), _ in ks if b > lo and a < hi)
        gaps_us = sorted(((b - a) / 1e3 for a, b in gaps), reverse=True)
        res[name] = {
            "wall_ms": round(wall / 1e6, 3),
            "kernel_dispatches": n_disp,
            "device_idle_pct": round(100.0 * (1 - busy / wall), 3) if wall else None,
            "loader_kernel_pct": round(100.0 * lbusy / wall, 3) if wall else None,
            "copy_busy_pct": round(100.0 * cbusy / wall, 3) if wall else None,
            "gaps_over_20us": sum(1 for g in gaps_us if g > 20),
            "longest_gaps_us": [round(g, 1) for g in gaps_us[:5]],
        }
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace_dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--names", default="bench.phase1,bench.phase2",
                    help="comma-separated roctx range names to analyse (bench_idle_sweep.py: sweep.p00,...)")
    a = ap.parse_args(argv)
    kernels = [r for p in _find(a.trace_dir, "kernel_trace.csv") for r in _rows(p)]
    copies = [r for p in _find(a.trace_dir, "memory_copy_trace.csv") for r in _rows(p)]
    markers = [r for p in _find(a.trace_dir, "marker_api_trace.csv") for r in _rows(p)]
    if not kernels or not markers:
        print(f"no kernel/marker trace under {a.trace_dir}", file=sys.stderr)
        return 1
    res = analyse(kernels, copies, markers, tuple(n for n in a.names.split(",") if n))
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
