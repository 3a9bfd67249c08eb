#!/usr/bin/env python3
"""Attribute the compute stream's idle gaps inside a roctx range of a rocprofv3 trace.

``tools/trace_idle.py`` measures how long the GPU had nothing resident; this tool asks WHY the
compute stream (the stream that ran the most kernel time in the range: the train step's) sat idle
between two of its kernels. Each gap longer than ``--min-us`` is put in one bucket:

* ``batch_kernel``: a loader kernel on another stream (the batch gather / collate) ran inside the
  gap (or ended within ``--slack-us`` of it) -- the compute stream waited for the batch (cross-stream
  event wait); ``batch_kernel_after_h2d_copy`` when an H2D copy also landed in the gap: the batch
  kernel itself had waited for its window's copy;
* ``h2d_copy``: an H2D copy ended inside the gap -- the batch's window was still in flight;
* ``host``: neither -- nothing on the device was pending, the host had not enqueued the next
  kernel yet (launch latency, a blocking host call).

Input: the directory given to ``rocprofv3 --kernel-trace --memory-copy-trace --marker-trace
--output-format csv -d DIR``. Output: one JSON object.
"""

from __future__ import annotations

import argparse
import bisect
import collections
import json
import sys

from trace_idle import LOADER_KERNELS, _find, _rows, _ts


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace_dir")
    ap.add_argument("--range", required=True, help="roctx range name (e.g. sweep.p00)")
    ap.add_argument("--min-us", type=float, default=2.0)
    ap.add_argument("--slack-us", type=float, default=3.0)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args(argv)

    kern = [r for f in _find(a.trace_dir, "kernel_trace.csv") for r in _rows(f)]
    copies = [r for f in _find(a.trace_dir, "memory_copy_trace.csv") for r in _rows(f)]
    marks = [r for f in _find(a.trace_dir, "marker_api_trace.csv") for r in _rows(f)]
    rng = [m for m in marks if m["Function"] == a.range]
    if not rng:
        print(json.dumps({"error": f"range {a.range!r} not found"}))
        return 1
    lo, hi = _ts(rng[0])
    inside = [r for r in kern if _ts(r)[1] > lo and _ts(r)[0] < hi]
    busy = collections.Counter()
    for r in inside:
        s, e = _ts(r)
        busy[(r["Agent_Id"], r["Queue_Id"])] += e - s
    compute_q = busy.most_common(1)[0][0]
    comp = sorted((_ts(r) + (r["Kernel_Name"],) for r in inside if (r["Agent_Id"], r["Queue_Id"]) == compute_q))
    loader = sorted(_ts(r) for r in inside if (r["Agent_Id"], r["Queue_Id"]) != compute_q
                    and any(k in r["Kernel_Name"] for k in LOADER_KERNELS))
    copy_ends = sorted(_ts(r)[1] for r in copies if r["Direction"].endswith("HOST_TO_DEVICE")
                       and _ts(r)[1] > lo and _ts(r)[0] < hi)

    def ends_in(ends, a0, b0):
        i = bisect.bisect_left(ends, a0)
        return i < len(ends) and ends[i] <= b0

    buckets = collections.Counter()
    counts = collections.Counter()
    after = collections.Counter()
    gaps = []
    slack = int(a.slack_us * 1000)
    for (s0, e0, _), (s1, e1, n1) in zip(comp, comp[1:]):
        g = s1 - e0
        if g < a.min_us * 1000:
            continue
        # a loader kernel running in the gap, or ending within the slack of its end (queues' clocks
        # differ by a few us): the compute stream waited for the batch; if an H2D copy landed in the
        # gap too, the batch kernel itself waited for its window's copy
        j = bisect.bisect_left(loader, (e0 - slack, 0))
        waited = any(a0 < s1 + slack and b0 > e0 for a0, b0 in loader[max(0, j - 4):j + 8])
        copy_late = ends_in(copy_ends, e0, s1 + slack)
        if waited and copy_late:
            b = "batch_kernel_after_h2d_copy"
        elif waited:
            b = "batch_kernel"
        elif copy_late:
            b = "h2d_copy"
        else:
            b = "host"
        buckets[b] += g
        counts[b] += 1
        after[n1[:60]] += g
        gaps.append((g, b, n1[:80]))
    wall = hi - lo
    out = {
        "range": a.range, "wall_ms": round(wall / 1e6, 3), "compute_queue": list(compute_q),
        "compute_kernels": len(comp),
        "gap_ms_by_cause": {k: round(v / 1e6, 4) for k, v in buckets.items()},
        "gap_count_by_cause": dict(counts),
        "gap_pct_of_wall_by_cause": {k: round(100.0 * v / wall, 3) for k, v in buckets.items()},
        "gap_ms_by_next_kernel": {k: round(v / 1e6, 4) for k, v in after.most_common(a.top)},
        "longest_gaps_us": [(round(g / 1e3, 1), b, n) for g, b, n in sorted(gaps, reverse=True)[: a.top]],
    }
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
