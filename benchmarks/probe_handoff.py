#!/usr/bin/env python3
"""What costs the compute stream idle time at a step boundary when each step consumes a batch built on
another stream? The loader's pattern, rebuilt piece by piece without the loader.

Every variant runs the same calibrated step (batch read + bf16 GEMM chain, ``CalibratedStep``) for
``--steps`` steps between ``ComputeIdleMeter`` events and reports the meter's idle %:

* ``held``: one batch, read every step (the idle sweep's floor);
* ``rotate``: ``--n-bufs`` batch buffers used round-robin, nothing else running;
* ``side_gather``: each buffer is (re)built by the gather kernel on a side stream one step ahead; the
  host waits for it (``Event.synchronize``, the loader's host hand-off) before enqueuing the step;
* ``side_gather_nowait``: the same without any hand-off (the side kernel only runs concurrently; the
  batch may be overwritten while read -- a timing probe, not a loader);
* ``side_gather_devwait``: the compute stream waits for the side event (device-side hand-off);
* ``side_idle``: the side stream records an event per step but runs no kernel, host waits on it;
* ``h2d_gather`` / ``h2d_gather_nowait`` / ``h2d_gather_devwait``: as ``side_gather*``, but each gather
  first waits (on the side stream) for a window-sized H2D copy issued for it on a copy stream -- the
  loader's copy -> gather dependency.

``--h2d`` adds the loader's copy traffic (a window-sized H2D copy per step on a copy stream) to every
variant. Output: one JSON line per variant.
"""

from __future__ import annotations

import argparse
import json
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--step-ms", type=float, default=2.7)
    ap.add_argument("--n-bufs", type=int, default=8)
    ap.add_argument("--h2d", action="store_true")
    ap.add_argument("--variants", default="held,rotate,side_idle,side_gather,side_gather_nowait,side_gather_devwait,"
                                          "h2d_gather,h2d_gather_nowait,h2d_gather_devwait")
    a = ap.parse_args(argv)
    import torch

    from ddl_amd import ops
    from ddl_amd.models.trainstep import CalibratedStep
    from ddl_amd.permutation import FeistelPermutation
    from ddl_amd.utils.tracing import ComputeIdleMeter, trace_range

    dev = torch.device("cuda", 0)
    B, shape = 256, (3, 224, 224)
    window = torch.randn((B,) + shape, device=dev).to(torch.bfloat16)
    bufs = [torch.empty_like(window) for _ in range(a.n_bufs)]
    for b in bufs:
        b.copy_(window)
    side = torch.cuda.Stream(dev, priority=-1)
    copy_s = torch.cuda.Stream(dev)
    nbytes = window.numel() * 2
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    landing = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    ring = [torch.empty_like(window) for _ in range(2)]
    ring_pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    ring_pinned.view(torch.bfloat16).copy_(window.view(-1).cpu())
    copy2 = torch.cuda.Stream(dev)
    step = CalibratedStep(dev, step_ms=a.step_ms)
    step.calibrate(window)

    def run(variant: str) -> dict:
        cur = torch.cuda.current_stream(dev)
        evs = [torch.cuda.Event() for _ in range(a.n_bufs)]

        cev = [torch.cuda.Event() for _ in range(a.n_bufs)]

        def build(j):  # batch j on the side stream
            src = window
            if variant.startswith("h2d"):  # its window lands by H2D first (two ring buffers, behind their reads)
                rb = ring[j % 2]
                copy2.wait_stream(side)
                with torch.cuda.stream(copy2):
                    rb.view(-1).view(torch.uint8).copy_(ring_pinned, non_blocking=True)
                    cev[j % a.n_bufs].record(copy2)
                side.wait_event(cev[j % a.n_bufs])
                src = rb
            with torch.cuda.stream(side):
                if variant != "side_idle":
                    ops.gather_rows(src, perm=FeistelPermutation(B, 1, j), base=0, n_rows=B, out=bufs[j % a.n_bufs])
                evs[j % a.n_bufs].record(side)

        side_v = variant.startswith("side") or variant.startswith("h2d")
        if side_v:
            build(0)
        for _ in range(5):
            step(bufs[0])
        torch.cuda.synchronize()
        meter = ComputeIdleMeter()
        with trace_range(f"probe.{variant}"):
            for i in range(a.steps):
                if variant == "held":
                    batch = bufs[0]
                elif variant == "rotate":
                    batch = bufs[i % a.n_bufs]
                else:
                    batch = bufs[i % a.n_bufs]
                    if variant in ("side_gather", "side_idle", "h2d_gather"):
                        evs[i % a.n_bufs].synchronize()
                    elif variant in ("side_gather_devwait", "h2d_gather_devwait"):
                        cur.wait_event(evs[i % a.n_bufs])
                    build(i + 1)
                meter.step_begin()
                if a.h2d:  # one window copy per step, paced by the step's begin event
                    copy_s.wait_event(meter._cur)
                    with torch.cuda.stream(copy_s):
                        landing.copy_(pinned, non_blocking=True)
                step(batch)
                meter.step_end()
            torch.cuda.synchronize()
        r = meter.result()
        return {"variant": variant, "h2d": a.h2d, "gpu_idle_pct": round(r["gpu_idle_pct"], 3),
                "busy_ms_per_step": round(r["busy_ms"] / max(1, r["steps"]), 4),
                "idle_us_per_step": round((r["wall_ms"] - r["busy_ms"]) * 1000 / max(1, r["steps"] - 1), 2)}

    for v in a.variants.split(","):
        run(v)  # warm
    for v in a.variants.split(","):
        print(json.dumps(run(v)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
