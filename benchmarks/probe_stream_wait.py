#!/usr/bin/env python3
"""Device-side cost of a cross-stream wait on MI355X (the loader's per-step batch hand-off).

The lookahead dispatch builds batch i+1 on the batch stream while step i runs, and the compute stream
waits for it with ``hipStreamWaitEvent`` before step i+1. This probe measures what that wait costs on
the compute stream's timeline when the awaited event has ALREADY completed, against the same loop
without it:

* ``none``: K iterations of [bf16 GEMM chain] on the compute stream;
* ``stale``: + a wait per iteration on one event recorded once on another stream, long complete;
* ``fresh``: + a small kernel on another stream each iteration, whose event the compute stream waits
  for (the loader's pattern: the kernel is enqueued one iteration ahead, so it completes long before
  the wait is reached);
* ``same``: + a wait on an event recorded on the compute stream itself;
* ``h2d_nowait`` / ``h2d_wait``: the loader's surroundings -- a 77 MB H2D copy per iteration on a copy
  stream and a device copy of the landed buffer on the side stream behind it -- without / with the
  compute stream waiting for that side-stream work each iteration.

Each variant prints the mean extra microseconds per iteration over ``none``.
"""

import argparse
import json
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--gemms", type=int, default=4)
    ap.add_argument("--m", type=int, default=4096)
    a = ap.parse_args(argv)
    import torch

    dev = torch.device("cuda", 0)
    x = torch.randn(a.m, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16) / 64
    out = torch.empty_like(x)
    side = torch.cuda.Stream(dev, priority=-1)
    small = torch.empty(1 << 20, device=dev)
    stale = torch.cuda.Event()
    with torch.cuda.stream(side):
        small.add_(1)
        stale.record(side)
    torch.cuda.synchronize()

    # the loader's pattern around the wait: H2D window copies on a copy stream, a gather of the landed
    # window on the side stream behind the copy, the compute stream waiting for the gather
    pinned = torch.empty(77 << 20, dtype=torch.uint8, pin_memory=True)
    hbm = [torch.empty(77 << 20, dtype=torch.uint8, device=dev) for _ in range(2)]
    batch = torch.empty(77 << 20, dtype=torch.uint8, device=dev)
    copy_s = torch.cuda.Stream(dev)

    def run(mode):
        cur = torch.cuda.current_stream(dev)
        if mode.startswith("h2d"):  # background copies + gathers, the compute stream waits (h2d_wait) or not
            cev = [torch.cuda.Event() for _ in range(4)]
            gev = [torch.cuda.Event() for _ in range(4)]

            def stage(j):
                with torch.cuda.stream(copy_s):
                    hbm[j % 2].copy_(pinned, non_blocking=True)
                    cev[j % 4].record(copy_s)
                with torch.cuda.stream(side):
                    side.wait_event(cev[j % 4])
                    batch.copy_(hbm[j % 2])
                    gev[j % 4].record(side)

            stage(0)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.iters):
                if mode == "h2d_wait":
                    cur.wait_event(gev[i % 4])
                stage(i + 1)
                for _ in range(a.gemms):
                    torch.mm(x, w, out=out)
            e.record()
            e.synchronize()
            torch.cuda.synchronize()
            return s.elapsed_time(e) * 1000 / a.iters
        evs = [torch.cuda.Event() for _ in range(4)]
        if mode == "fresh":  # one iteration ahead, as the loader's lookahead
            with torch.cuda.stream(side):
                small.add_(1)
                evs[0].record(side)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(a.iters):
            if mode == "stale":
                cur.wait_event(stale)
            elif mode == "fresh":
                cur.wait_event(evs[i % 4])
                with torch.cuda.stream(side):
                    small.add_(1)
                    evs[(i + 1) % 4].record(side)
            elif mode == "same":
                ev = evs[i % 4]
                ev.record(cur)
                cur.wait_event(ev)
            for _ in range(a.gemms):
                torch.mm(x, w, out=out)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1000 / a.iters

    modes = ("none", "stale", "fresh", "same", "h2d_nowait", "h2d_wait")
    for mode in modes:
        run(mode)  # warm
    res = {m: run(m) for m in modes + ("none",)}
    base = res["none"]
    out = {"probe": "cross-stream wait cost on the compute stream", "iter_us_none": round(base, 2)}
    for m in ("stale", "fresh", "same", "h2d_nowait", "h2d_wait"):
        out[f"extra_us_{m}"] = round(res[m] - base, 2)
    out["extra_us_wait_under_h2d"] = round(res["h2d_wait"] - res["h2d_nowait"], 2)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
