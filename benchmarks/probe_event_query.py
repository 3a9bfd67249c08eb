#!/usr/bin/env python3
"""Does hipEventQuery report a pending copy / kernel as complete? (round-3 diagnostic)

The stager's adaptive copy policy asked "has the last copy on stream 0 retired?" with hipEventQuery and
found it retired for 192 of 199 copies while two copies overlapped under strict alternation on the same
box (archive/profiles/r3_copy_policy). This probe records events right after work that takes milliseconds and
queries them at once:

* after a 1 GiB pinned H2D copy (SDMA) on a side stream;
* after the same copy queued behind a device-side wait on an event that is still pending;
* after a long kernel chain on a side stream;
* for an event that was never recorded (HIP reports success for it).

Each line reports the query result right after the record, and after a synchronize.
"""

import json
import time

import torch


def main() -> int:
    dev = torch.device("cuda", 0)
    n = 1 << 30
    src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out = []

    def rec(name, ev, t_enq):
        q0 = ev.query()
        t0 = time.perf_counter()
        ev.synchronize()
        out.append({"case": name, "query_right_after_record": q0,
                    "ms_until_complete": round(1e3 * (time.perf_counter() - t0), 3),
                    "ms_enqueue": round(1e3 * t_enq, 3), "query_after_sync": ev.query()})

    for flags in ((False, False), (True, True)):
        tag = f"blocking={flags[0]},timing={flags[1]}"
        dst.copy_(src)  # warm the engine
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            dst.copy_(src, non_blocking=True)
            ev = torch.cuda.Event(blocking=flags[0], enable_timing=flags[1])
            ev.record()
        rec(f"h2d_1GiB [{tag}]", ev, time.perf_counter() - t)

        t = time.perf_counter()
        with torch.cuda.stream(s2):
            for _ in range(20):
                torch.mm(a, a)
            gate = torch.cuda.Event(blocking=flags[0], enable_timing=flags[1])
            gate.record()
        s1.wait_event(gate)
        with torch.cuda.stream(s1):
            dst.copy_(src, non_blocking=True)
            ev = torch.cuda.Event(blocking=flags[0], enable_timing=flags[1])
            ev.record()
        rec(f"h2d_behind_pending_wait [{tag}]", ev, time.perf_counter() - t)

        t = time.perf_counter()
        with torch.cuda.stream(s2):
            for _ in range(20):
                torch.mm(a, a)
            ev = torch.cuda.Event(blocking=flags[0], enable_timing=flags[1])
            ev.record()
        rec(f"gemm_chain [{tag}]", ev, time.perf_counter() - t)
        torch.cuda.synchronize()

    never = torch.cuda.Event()
    out.append({"case": "never_recorded", "query": never.query()})
    for o in out:
        print(json.dumps(o), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
