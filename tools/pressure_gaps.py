#!/usr/bin/env python3
"""Where the GPU idle of ``bench.py``'s pressure phase (r = 0.9) sits, per step (GPU box, one rank).

The headline loader (3 stamp producers, 256-sample bf16 windows, device shuffle) feeds a ``CalibratedStep``
sized at ``--ratio`` x the measured feed. Per step this records the device gap in front of the step (end of
step k-1 to start of step k on the compute stream), the host time spent in ``dl[i]``, in ``mark`` and in
enqueueing the step, and whether the GPU had already drained step k-1 when the host enqueued step k
(``late``: the gap is the host's). Prints one JSON line per ``--dispatch`` with the gap percentiles, the idle
split between late and not-late steps, and the host context of the largest gaps.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(args, dispatch: str) -> dict:
    import torch

    import ddl_amd
    from ddl_amd import Marker, ops
    from ddl_amd.models.producers import ImageWindowProducer
    from ddl_amd.models.trainstep import CalibratedStep
    from ddl_amd.utils.tracing import ComputeIdleMeter

    if args.block_mb:  # output blocks of the batch engine and of the indexed loaders
        from ddl_amd.engine_dispatch import NativeDispatchMixin
        from ddl_amd.resident import PrefetchedIndexedLoader

        NativeDispatchMixin.engine_block_bytes = PrefetchedIndexedLoader.block_bytes = args.block_mb << 20
    if args.no_record_stream:  # A/B only: batches' allocator blocks are then unprotected across streams
        torch.Tensor.record_stream = lambda self, stream: None
    with ddl_amd.start(n_producers=3 if args.path == "window" else 0) as (env, conn):
        dev = torch.device(env.device)
        spare = [torch.cuda.Stream(dev) for _ in range(args.spare_streams)]  # shifts the stream -> HW queue map
        host = {"get": [], "mark": [], "step": []}
        if args.path == "zero_copy":
            from ddl_amd.zerocopy import ZeroCopyLoader

            src = torch.empty((4096, 3, 224, 224), dtype=torch.bfloat16).pin_memory()
            src.view(4096, -1)[:, 0] = torch.arange(4096, dtype=torch.bfloat16)
            dl = ZeroCopyLoader(src, 256, env, seed=0, out_dtype=torch.bfloat16, device=dev,
                                max_blocks=args.zc_blocks, handoff="host")
        else:
            dl = ddl_amd.DistributedDataLoader(
                ImageWindowProducer(256, (3, 224, 224), "bfloat16", seed=0, refill="stamp"), 256, conn, 10 ** 6,
                env=env, device=dev, output=ddl_amd.OutputSpec(dtype=torch.bfloat16),
                order=ddl_amd.OrderSpec(shuffle="device", seed=0),
                staging=ddl_amd.StagingSpec(prefetch_depth=args.depth, native_dispatch=dispatch,
                                            copy_timing=args.copy_timing))

        def zc_batches():
            while True:
                t0 = time.perf_counter()
                for x in dl:
                    host["get"].append(time.perf_counter() - t0)
                    host["mark"].append(0.0)
                    yield (x,)
                    t0 = time.perf_counter()

        def batches():
            while True:
                for i in range(len(dl)):
                    t0 = time.perf_counter()
                    x = dl[i]
                    t1 = time.perf_counter()
                    host["get"].append(t1 - t0)
                    yield x
                    t2 = time.perf_counter()
                    dl.mark(Marker.END_OF_BATCH)
                    host["mark"].append(time.perf_counter() - t2)
                dl.mark(Marker.END_OF_EPOCH)

        it = zc_batches() if args.path == "zero_copy" else batches()
        acc = ops.ChecksumAccumulator(dev)
        for _ in range(50):
            acc.add(next(it)[0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            acc.add(next(it)[0])
        torch.cuda.synchronize()
        feed = 256 * 200 / (time.perf_counter() - t0)
        step = CalibratedStep(dev, step_ms=1000.0 * 256 / (args.ratio * feed))
        step.calibrate(next(it)[0])
        for _ in range(2):  # re-size from the busy time on the loader's batches, as bench.py's pressure phase
            ends = []
            for _ in range(40):
                (x,) = next(it)
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                step(x)
                s1.record()
                ends.append((s0, s1))
            torch.cuda.synchronize()
            step.tune(sum(s0.elapsed_time(s1) for s0, s1 in ends) / len(ends))
        for k in host:
            host[k].clear()
        n = args.steps
        late = [False] * n
        if args.meter == "bench":  # bench.py's ComputeIdleMeter: a fresh pair of timing events per step
            meter = ComputeIdleMeter()
            for k in range(n):
                (x,) = next(it)
                t0 = time.perf_counter()
                meter.step_begin()
                step(x)
                meter.step_end()
                host["step"].append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            evs = meter._pairs
        else:  # events created up front; "late" probes query step k-1's end event before step k is enqueued
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
            for k in range(n):
                (x,) = next(it)
                t0 = time.perf_counter()
                if k > 0 and args.meter == "late":
                    late[k] = evs[k - 1][1].query()  # the GPU already ran out of step k-1 when step k was enqueued
                evs[k][0].record()
                step(x)
                evs[k][1].record()
                host["step"].append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        st = dl.stats()
        dl.close()
        del dl
    busy = [s.elapsed_time(e) for s, e in evs]
    gaps = [1000.0 * evs[k - 1][1].elapsed_time(evs[k][0]) for k in range(1, n)]
    wall = evs[0][0].elapsed_time(evs[-1][1])
    g_sorted = sorted(gaps)

    def pct(q):
        return round(g_sorted[min(len(g_sorted) - 1, int(q * len(g_sorted)))], 1)

    late_gap = sum(g for k, g in enumerate(gaps, 1) if late[k])
    # host context of the largest gaps: step k's own get / mark / enqueue and the previous step's
    get, mark, enq = host["get"][-n:], host["mark"][-n:], host["step"]
    top = sorted(range(1, n), key=lambda k: -gaps[k - 1])[:args.top]
    ctx = [{"k": k, "gap_us": round(gaps[k - 1], 1), "late": late[k],
            "get_us": [round(1e6 * get[j], 1) for j in range(max(0, k - 2), k + 1)],
            "mark_us": [round(1e6 * mark[j], 1) for j in range(max(0, k - 2), min(len(mark), k + 1))],
            "enqueue_us": round(1e6 * enq[k], 1)} for k in top]
    return {"dispatch": dispatch, "meter": args.meter, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "spare_streams": len(spare),
            "depth": args.depth, "copy_timing": args.copy_timing, "steps": n,
            "feed": round(feed, 1), "ratio_measured": round(1000.0 * 256 / (sum(busy) / n) / feed, 3),
            "idle_pct": round(100.0 * (1.0 - sum(busy) / wall), 3),
            "gaps_us": {"p50": pct(0.5), "p90": pct(0.9), "p99": pct(0.99), "max": round(g_sorted[-1], 1)},
            "late_steps": sum(late), "late_share_of_gap": round(late_gap / max(1e-9, sum(gaps)), 3),
            "host_us_p50": {k: round(1e6 * sorted(v)[len(v) // 2], 1) for k, v in (("get", get), ("mark", mark),
                                                                                  ("enqueue", enq))},
            "top": ctx, "engine": st.get("native_dispatch"), "path": args.path,
            "record_stream": not args.no_record_stream, "block_mb": args.block_mb,
            "zc_host_waits": st.get("host_waits")}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--dispatch", default="lookahead")
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--ratio", type=float, default=0.9)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--copy-timing", action="store_true")
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--path", default="window", choices=["window", "zero_copy"])
    ap.add_argument("--zc-blocks", type=int, default=None)
    ap.add_argument("--no-record-stream", action="store_true")
    ap.add_argument("--block-mb", type=int, default=0, help="output block size (default: the library's)")
    ap.add_argument("--meter", default="late", choices=["late", "plain", "bench"],
                    help="late: events made up front + a query of step k-1's end per step; plain: without the "
                         "query; bench: bench.py's ComputeIdleMeter (events made per step)")
    ap.add_argument("--spare-streams", type=int, default=0,
                    help="idle HIP streams created before the loader's (HIP maps streams round-robin onto "
                         "GPU_MAX_HW_QUEUES hardware queues)")
    args = ap.parse_args()
    for d in args.dispatch.split(","):
        print(json.dumps(run(args, d)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
