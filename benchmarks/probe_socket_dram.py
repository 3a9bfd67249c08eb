#!/usr/bin/env python3
"""Host-DRAM headroom of one socket: can it feed 4 GPUs' H2D plus their producers' full refills?

At N=8 four ranks share each socket (`utils/numa.py` binds a rank to its GPU's node). Each rank's feed
reads ~56 GB/s of pinned windows out of that node's DRAM (the SDMA engines' H2D), and with full-refill
producers (``bench.py --refill full``, the reference's every-round window rewrite,
``/root/reference/ddl/datapusher.py:151-166``) each delivered window is also rewritten on the host:
one read of the pristine rows plus one write of the window. Per socket that is

    stamp refills:  4 x 56 GB/s DMA reads                                   ~224 GB/s
    full refills:   4 x (56 DMA read + 56 refill read + 56 refill write)     ~672 GB/s

The one-GPU box cannot run 4 GPUs, so this probe emulates one socket's share on the GPU's NUMA node:

* ``h2d``: the real H2D of this GPU (two copy streams, 77 MB windows from node-local pinned memory);
* ``dma_emul``: host threads streaming READS over node-local buffers, standing in for the other
  3 GPUs' DMA reads (read-only, like an SDMA engine pulling a window);
* ``refill``: the producers' full refill (``gather_rows`` of a random permutation, the native host pool
  the producers use), i.e. read + write traffic.

Phases (each ``--seconds`` long): every component alone, then combinations, up to the full socket load.
For every phase it reports each component's GB/s and the total DRAM traffic (reads + writes). The
prediction for N=8 follows from whether the full-load phase holds every component at its target:
``--target-gbps`` (default 56) per GPU for DMA and per rank for refills.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np


def _parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--window-mb", type=float, default=77.07, help="bytes per window (256 x 3x224x224 bf16)")
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--dma-threads", type=int, default=6, help="host read threads emulating 3 more GPUs' DMA")
    ap.add_argument("--refill-threads", type=int, default=8, help="threads of the refill host pool (4 ranks)")
    ap.add_argument("--target-gbps", type=float, default=56.0)
    ap.add_argument("--stream-stores", default="on", choices=["on", "off"],
                    help="refill copies with non-temporal stores (the runtime default) or plain memcpy")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


class _Loop:
    """Run ``fn`` back to back in a thread until stopped; count bytes."""

    def __init__(self, fn, nbytes: int):
        self.fn, self.nbytes = fn, nbytes
        self.count = 0
        self._stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            self.fn()
            self.count += 1

    def start(self):
        self.t0 = time.perf_counter()
        self.t.start()
        return self

    def stop(self) -> float:
        self._stop.set()
        self.t.join()
        return self.count * self.nbytes / (time.perf_counter() - self.t0) / 1e9


def main(argv=None) -> int:
    a = _parse(argv)
    import torch

    from ddl_amd import _native
    from ddl_amd.utils.numa import bind_to_gpu_numa, gpu_numa_node

    node = bind_to_gpu_numa(0, 1)
    cpus = sorted(os.sched_getaffinity(0))
    rt = _native.runtime()
    rt.set_stream_stores(a.stream_stores == "on")
    wb = int(a.window_mb * 1e6) // 4096 * 4096
    dev = torch.device("cuda", 0)

    # --- buffers, first touched by this (node-bound) process
    pinned = [torch.empty(wb, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    for p in pinned:
        p.fill_(1)
    dst = [torch.empty(wb, dtype=torch.uint8, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    row = 301056
    n_rows = wb // row
    base = torch.empty(n_rows * row, dtype=torch.uint8)
    base.fill_(3)
    win = torch.empty(n_rows * row, dtype=torch.uint8)
    win.fill_(0)
    reads = [np.ones(wb // 8, dtype=np.uint64) for _ in range(max(1, a.dma_threads))]
    nodes = {"pinned": list(rt.memory_nodes(pinned[0].data_ptr(), wb, 16)),
             "refill": list(rt.memory_nodes(win.data_ptr(), win.numel(), 16)),
             "dma_emul": list(rt.memory_nodes(reads[0].ctypes.data, reads[0].nbytes, 16))}
    rng = np.random.default_rng(0)

    def h2d():
        for s, d, p in zip(streams, dst, pinned):
            with torch.cuda.stream(s):
                d.copy_(p, non_blocking=True)
        for s in streams:
            s.synchronize()

    def refill():
        rt.gather_rows(win.data_ptr(), base.data_ptr(), row, rng.permutation(n_rows).astype(np.int64), n_rows,
                       a.refill_threads)

    def reader(i):
        return lambda: reads[i].sum()  # numpy releases the GIL in the reduction loop

    h2d()  # warm the copy engines
    refill()

    def phase(name, h2d_on, dma_on, refill_on):
        loops = {}
        if h2d_on:
            loops["h2d"] = _Loop(h2d, 2 * wb)
        if refill_on:
            loops["refill"] = _Loop(refill, n_rows * row)
        dma = [_Loop(reader(i), wb) for i in range(a.dma_threads)] if dma_on else []
        for lp in [*loops.values(), *dma]:
            lp.start()
        time.sleep(a.seconds)
        out = {k: round(v.stop(), 2) for k, v in loops.items()}
        if dma:
            out["dma_emul"] = round(sum(lp.stop() for lp in dma), 2)
        # DRAM traffic: H2D and emulated DMA read once; a refill reads the pristine row and writes the window
        out["dram_total"] = round(out.get("h2d", 0) + out.get("dma_emul", 0) + 2 * out.get("refill", 0), 2)
        out["phase"] = name
        print(json.dumps(out), flush=True)
        return out

    res = [phase("h2d", True, False, False),
           phase("dma_emul", False, True, False),
           phase("refill", False, False, True),
           phase("h2d+dma_emul (stamp socket)", True, True, False),
           phase("h2d+refill", True, False, True),
           phase("h2d+dma_emul+refill (full socket)", True, True, True)]
    t = a.target_gbps
    full = res[-1]
    summary = {
        "probe": "socket DRAM headroom (one socket's share of an 8-rank job, emulated on the GPU's node)",
        "gpu_numa_node": gpu_numa_node(0), "bound_node": node, "cpus": len(cpus),
        "stream_stores": bool(rt.stream_stores()),
        "page_nodes": nodes,
        "demand_gbps": {"stamp": 4 * t, "full": 12 * t},
        "target_per_gpu_gbps": t,
        "phases": res,
        "h2d_drop_under_full_load_pct": round(100.0 * (1 - full["h2d"] / max(1e-9, res[0]["h2d"])), 2),
        "max_dram_total_gbps": max(r["dram_total"] for r in res),
    }
    print(json.dumps(summary), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(summary) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
