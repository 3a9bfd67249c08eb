#!/usr/bin/env python3
"""GPU idle % under loader pressure: a calibrated step swept across the feed rate.

``bench.py``'s phase 2 measures idle % behind a PatchMLP step that runs ~4x
slower than the feed, which says nothing about overlap when the loader is the
bottleneck. Here:

1. phase 1 measures the loader's feed rate ``F`` (samples/s; the consumer only
   checksums every delivered byte), as in ``bench.py``;
2. for each ratio ``r`` a ``CalibratedStep`` (batch read + a bf16 GEMM chain
   sized on this GPU) is built whose step capacity is ``C = r * F``, i.e. a
   GPU step time of ``B / (r * F)``; the loop runs it on the loader's batches
   and measures the compute stream's idle % with HIP events
   (``ComputeIdleMeter``) and the achieved samples/s.

If the loader overlaps perfectly, a step FASTER than the feed (``r > 1``) is
starved exactly by the missing feed: ``idle = 1 - F / C_measured`` where
``C_measured = B / (busy per step)``; a step slower than the feed (``r <= 1``)
never waits: ``idle = 0``. So the prediction is ``max(0, 1 - F / C_measured)``
and each point reports it next to the measurement. Every point is bracketed
by a roctx range ``sweep.pNN`` so ``tools/trace_idle.py --names`` can
cross-check it from a rocprofv3 kernel trace.

Families: ``images`` (config 2: 3x224x224, bf16 source or ``--source-dtype
uint8`` cast + normalised on the device) and ``tokens`` (config 4: seq_len
4096, ragged H2D + on-device pack). One GPU; prints one JSON line per point
and a summary line.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

RATIOS = (0.5, 0.75, 0.9, 1.0, 1.1, 1.25, 1.5, 2.0)


def _parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--family", default="images", choices=["images", "tokens"])
    ap.add_argument("--source-dtype", default="bfloat16", choices=["bfloat16", "uint8"])
    ap.add_argument("--ratios", default=",".join(str(r) for r in RATIOS))
    ap.add_argument("--step-ms", default=None,
                    help="absolute step times in ms instead of ratios to the measured feed (compares loader variants "
                         "whose feeds differ at the same step: a ratio to each one's own feed would not)")
    ap.add_argument("--feed-steps", type=int, default=300)
    ap.add_argument("--steps", type=int, default=150, help="timed steps per sweep point")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=None,
                    help="images: 256 samples; tokens: 2048 sequences (a GPU step long enough to dominate the "
                         "per-batch host cost)")
    ap.add_argument("--window", type=int, default=256)
    ap.add_argument("--producers", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None, help="HBM prefetch depth (windows); default: the loader's")
    ap.add_argument("--feed-keepalive", action="store_true",
                    help="keep the GPU busy with low-priority GEMMs while the feed rate F is measured (a GPU idling "
                         "between loader kernels runs the host-latency-bound token path slower than under a step)")
    ap.add_argument("--tokens-k", type=int, default=8,
                    help="tokens: global batches per window (k-batch windows amortise the per-window host path)")
    ap.add_argument("--floor", action="store_true",
                    help="after each point, run the same step on one held batch (no loader) with the same meter: "
                         "the idle the measurement itself shows without any loader work (floor_idle_pct)")
    ap.add_argument("--floor-traffic", action="store_true",
                    help="images: also run the floor loop with the loader's device traffic and no loader hand-off: "
                         "per step one window H2D copy (two copy streams) and a device copy of it on a side stream, "
                         "paced by the step's begin event; nothing waits on the compute stream "
                         "(floor_traffic_idle_pct)")
    ap.add_argument("--prealloc-gb", type=float, default=0.0,
                    help="grow the caching allocator's pool on the loader's batch stream by this many GB before the "
                         "sweep, so output blocks come from cached memory instead of new hipMalloc segments while the "
                         "host runs ahead of the GPU")
    ap.add_argument("--dispatch", default="auto", help="native_dispatch of the image loader (auto / inline / "
                                                         "lookahead / python)")
    ap.add_argument("--tune-passes", type=int, default=2,
                    help="per point: re-size the calibrated step this many times from its busy time measured on the "
                         "loader's batches (the isolated calibration runs at other clocks and without the loader's "
                         "memory traffic, and landed 0.75 at a measured 0.91-0.94)")
    ap.add_argument("--tune-steps", type=int, default=30)
    ap.add_argument("--read", default="all", choices=["all", "ids"],
                    help="tokens: the consumer reads every tensor of the batch (all) or only input_ids (ids, as "
                         "bench_tokens.py's feed phase)")
    ap.add_argument("--max-ahead", type=int, default=None, help="DistributedDataLoader(max_ahead=) (A/B; default 16)")
    ap.add_argument("--lead-diag", action="store_true",
                    help="per step: how many enqueued steps the GPU had not finished when the host enqueued this one "
                         "(0 = the host is late: the compute stream ran dry), and the host time of each fetch")
    ap.add_argument("--stream-copies", action="store_true",
                    help="A/B: window copies on HIP copy streams instead of straight onto SDMA engines through ROCr")
    ap.add_argument("--batch-priority", default="high", choices=["high", "normal"],
                    help="priority of the loader's batch stream (A/B; the library uses high)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--markers", action="store_true", help="roctx markers around each step's fetch (trace_gaps)")
    return ap.parse_args(argv)


def _image_loader(a, env, conn, n_steps):
    import torch

    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.models.producers import ImageWindowProducer

    B = a.batch or 256
    norm = None
    if a.source_dtype == "uint8":
        norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225], "layout": "chw"}
    n_epochs = math.ceil(n_steps / max(1, a.window // B)) + 2
    dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(a.window, (3, 224, 224), a.source_dtype, refill="stamp"), B,
                                       conn, n_epochs, env=env, device=torch.device(env.device),
                                       **{"prefetch_depth": a.depth} if a.depth else {},
                                       **{"max_ahead": a.max_ahead} if a.max_ahead is not None else {},
                                       output=ddl_amd.OutputSpec(dtype=torch.bfloat16, normalize=norm),
                                       staging=ddl_amd.StagingSpec(
                                           native_dispatch=a.dispatch != "python" and a.dispatch, copy_timing=True),
                                       order=ddl_amd.OrderSpec(shuffle="device"))

    def gen():
        while True:
            for i in range(len(dl)):
                yield dl[i]
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)

    return dl, gen(), B, "samples"


class _Traffic:
    """The loader's device traffic without the loader: per step, one window-sized H2D copy from pinned memory
    into a 2-buffer HBM ring (alternating copy streams, as the stager) and a device copy of the landed buffer on
    a side stream behind it (the batch gather's bytes). Each copy waits for the step's begin event, so the
    traffic is spread over the steps as the loader's is; the compute stream itself never waits for it."""

    def __init__(self, dev, nbytes: int):
        import torch

        self.torch = torch
        self.pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.ring = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.copy = [torch.cuda.Stream(dev) for _ in range(2)]
        self.side = torch.cuda.Stream(dev)
        self.j = 0

    def step(self, begin_event) -> None:
        torch = self.torch
        j = self.j
        self.j += 1
        cs = self.copy[j % 2]
        cs.wait_event(begin_event)
        with torch.cuda.stream(cs):
            self.ring[j % 2].copy_(self.pinned, non_blocking=True)
        self.side.wait_stream(cs)
        with torch.cuda.stream(self.side):
            self.out.copy_(self.ring[j % 2])
        cs.wait_stream(self.side)  # the ring buffer is re-filled only after its device copy


def _token_loader(a, env, conn, n_steps, src):
    import ddl_amd
    from ddl_amd.models.tokens import TokenBatchProducer

    B = a.batch or 2048
    n_epochs = n_steps // (src.n // B) + 2
    dl = ddl_amd.DistributedDataLoader(
        TokenBatchProducer(src, B, 4096, "pack", pack_order="ffd", host_threads=4,
                                                          batches_per_window=a.tokens_k), B, conn, n_epochs, env=env,
        auto_mark=True, **{"prefetch_depth": a.depth} if a.depth else {}, output=ddl_amd.OutputSpec(collate="tokens"),
        staging=ddl_amd.StagingSpec(n_slots=2, copy_timing=True), order=ddl_amd.OrderSpec(mode="indexed"))

    def gen():
        while True:
            yield from dl

    return dl, gen(), B, "sequences"


def main(argv=None) -> int:
    a = _parse(argv)
    import torch

    import ddl_amd
    from ddl_amd import ops
    from ddl_amd.models.trainstep import CalibratedStep
    from ddl_amd.utils.tracing import ComputeIdleMeter, trace_range

    ratios = [float(x) for x in a.ratios.split(",") if x]
    if a.stream_copies:
        from ddl_amd import staging as _stg

        _stg.DIRECT_DMA = False
    if a.batch_priority == "normal":  # A/B: the loader's batch stream at normal priority
        import ddl_amd.dataloader as _dl
        from ddl_amd.utils import streams as _streams

        _streams.batch_stream = _dl.streams.batch_stream = lambda device: torch.cuda.Stream(device)
    host_marks = a.markers
    n_steps = a.warmup + 2 * a.feed_steps + len(ratios) * (a.steps + a.warmup + a.tune_passes * a.tune_steps + 30)
    src = None
    if a.family == "tokens":
        from ddl_amd.models.tokens import SharedTokenSource

        from ddl_amd.utils.numa import gpu_numa_node

        src = SharedTokenSource.synthetic(f"ddl_amd_sweep_{os.getpid()}", 8192, 256, 4096, seed=1)
        src.bind_to_node(gpu_numa_node(0))  # next to the producers (bound to the GPU's node)
    # tokens: 6 producers x 4 gather threads x 2 slots -- the host-bound feed then has headroom, so it is
    # consumer-bound and stable from run to run (archive/profiles/r3_tokens)
    producers = a.producers or (3 if a.family == "images" else 6)
    points = []
    try:
        with ddl_amd.start(n_producers=producers) as (env, conn):
            if a.family == "images":
                dl, it, B, unit = _image_loader(a, env, conn, n_steps)
            else:
                dl, it, B, unit = _token_loader(a, env, conn, n_steps, src)
            dev = torch.device(env.device)
            acc = ops.ChecksumAccumulator(dev)

            keys = ("input_ids",) if a.read == "ids" and a.family == "tokens" else None

            def read(batch):
                if isinstance(batch, dict):
                    batch = batch.values() if keys is None else [batch[k] for k in keys]
                for t in batch:
                    if isinstance(t, torch.Tensor):
                        acc.add(t)

            # ---- phase 1: feed rate F, measured twice; the faster pass counts (a first pass can still
            # carry one-time costs -- first touch of source pages, allocator growth -- and an
            # underestimated F shows up as steps achieving more than the "feed")
            for _ in range(a.warmup):
                read(next(it))
            feeds = []
            keep = None
            if a.feed_keepalive:  # GEMMs on a low-priority stream keep the GPU busy (clocks up) during the feed
                keep = (torch.cuda.Stream(dev, priority=0), torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16))
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                with trace_range(f"sweep.feed{rep}"):
                    for k in range(a.feed_steps):
                        if keep is not None and k % 8 == 0:
                            with torch.cuda.stream(keep[0]):
                                for _ in range(8):
                                    torch.mm(keep[1], keep[1])
                        read(next(it))
                    torch.cuda.synchronize()
                feeds.append(B * a.feed_steps / (time.perf_counter() - t0))
            feed = max(feeds)
            print(json.dumps({"family": a.family, "feed_per_s": round(feed, 1), "feed_passes": [round(f, 1) for f in feeds],
                              "unit": unit}), flush=True)

            traffic = None
            if a.floor_traffic and a.family == "images":
                traffic = _Traffic(dev, a.window * 3 * 224 * 224 * (2 if a.source_dtype == "bfloat16" else 1))

            if a.prealloc_gb > 0 and getattr(dl, "_batch_stream", None) is not None:
                with torch.cuda.stream(dl._batch_stream):
                    blob = torch.empty(int(a.prealloc_gb * (1 << 30)), dtype=torch.uint8, device=dev)
                del blob

            # ---- sweep
            step_ms_list = [float(x) for x in a.step_ms.split(",")] if a.step_ms else None
            if step_ms_list:
                ratios = [1000.0 * B / (ms * feed) for ms in step_ms_list]
            for i, r in enumerate(ratios):
                step = CalibratedStep(dev, step_ms=step_ms_list[i] if step_ms_list else 1000.0 * B / (r * feed),
                                      read_keys=keys)
                step.calibrate(next(it))
                for _ in range(a.warmup):
                    step(next(it))
                for _ in range(a.tune_passes):  # re-size the step from its busy time in this very loop
                    tm = ComputeIdleMeter()
                    for _ in range(a.tune_steps):
                        batch = next(it)
                        tm.step_begin()
                        step(batch)
                        tm.step_end()
                    torch.cuda.synchronize()
                    tr = tm.result()
                    step.tune(tr["busy_ms"] / max(1, tr["steps"]))
                meter = ComputeIdleMeter()
                nd0 = dl.stats().get("native_dispatch") or {}
                seg0 = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                t2 = time.perf_counter()
                with trace_range(f"sweep.p{i:02d}"):
                    leads, fetch_us = [], []
                    for k in range(a.steps):
                        tf = time.perf_counter()
                        if host_marks:  # --markers: the host's mark + get per step, for trace_gaps
                            with trace_range("sweep.get"):
                                batch = next(it)
                        else:
                            batch = next(it)
                        if a.lead_diag:
                            fetch_us.append(1e6 * (time.perf_counter() - tf))
                            # how many enqueued steps the GPU has not finished yet when this one is enqueued
                            pairs, lead = meter._pairs, 0
                            for j in range(len(pairs) - 1, max(-1, len(pairs) - 33), -1):
                                if pairs[j][1].query():
                                    break
                                lead += 1
                            leads.append(lead)
                        meter.step_begin()
                        step(batch)
                        meter.step_end()
                    e1.record()
                    torch.cuda.synchronize()
                t3 = time.perf_counter()
                seg1 = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)
                res = meter.result()
                busy_per_step = res["busy_ms"] / max(1, res["steps"])
                cap = 1000.0 * B / busy_per_step  # measured step capacity C
                pred = 100.0 * max(0.0, 1.0 - feed / cap)
                pt = {"point": f"sweep.p{i:02d}", "ratio_target": r, "step_ms_target": round(step.step_ms, 4),
                      "gemm_reps": step.reps, "gemm_rows": step.a.shape[0], "gemm_tail_rows": step.tail_rows,
                      "busy_ms_per_step": round(busy_per_step, 4),
                      "step_capacity_per_s": round(cap, 1), "ratio_measured": round(cap / feed, 3),
                      "achieved_per_s": round(B * a.steps / (t3 - t2), 1),
                      "gpu_idle_pct": round(res["gpu_idle_pct"], 3), "predicted_idle_pct": round(pred, 3),
                      "error_pp": round(res["gpu_idle_pct"] - pred, 3),
                      "allocator_segments_created": seg1 - seg0, "gaps_us": res.get("gaps_us")}
                if getattr(dl, "_stager", None) is not None:
                    pt["copies"] = dl._stager.copy_summary(e0, e1)
                if a.lead_diag and leads:
                    import numpy as _np

                    pt["host_lead_steps"] = {"p10": float(_np.percentile(leads, 10)), "p50": float(_np.median(leads)),
                                             "p90": float(_np.percentile(leads, 90)),
                                             "at_0": int(sum(1 for x in leads if x == 0))}
                    pt["fetch_us"] = {"p50": round(float(_np.median(fetch_us)), 1),
                                      "p90": round(float(_np.percentile(fetch_us, 90)), 1),
                                      "max": round(max(fetch_us), 1)}
                if a.floor:  # the same step on one held batch, no loader calls: the meter's own floor
                    fm = ComputeIdleMeter()
                    torch.cuda.synchronize()
                    with trace_range(f"sweep.floor{i:02d}"):
                        for _ in range(a.steps):
                            fm.step_begin()
                            step(batch)
                            fm.step_end()
                        torch.cuda.synchronize()
                    fr = fm.result()
                    pt["floor_idle_pct"], pt["floor_gaps_us"] = round(fr["gpu_idle_pct"], 3), fr.get("gaps_us")
                    pt["error_vs_floor_pp"] = round(res["gpu_idle_pct"] - max(pred, pt["floor_idle_pct"]), 3)
                if traffic is not None:  # the same floor loop, with the loader's copies running beside it
                    tm = ComputeIdleMeter()
                    torch.cuda.synchronize()
                    with trace_range(f"sweep.traffic{i:02d}"):
                        for _ in range(a.steps):
                            tm.step_begin()
                            traffic.step(tm._cur)
                            step(batch)
                            tm.step_end()
                        torch.cuda.synchronize()
                    tr = tm.result()
                    pt["floor_traffic_idle_pct"] = round(tr["gpu_idle_pct"], 3)
                    pt["floor_traffic_busy_ms_per_step"] = round(tr["busy_ms"] / max(1, tr["steps"]), 4)
                st1 = dl.stats()
                nd1 = st1.get("native_dispatch") or {}
                if "run_ahead" in st1:
                    pt["run_ahead"] = st1["run_ahead"]
                if nd1:  # per point: batches built ahead (lookahead hits), batches the compute stream waited for
                    pt["dispatch"] = {"mode": nd1.get("mode"),
                                      **{k: nd1.get(k, 0) - nd0.get(k, 0)
                                         for k in ("batches", "lookahead_hits", "compute_waits", "ready_host_waits")}}
                points.append(pt)
                print(json.dumps(pt), flush=True)
            stats = dl.stats()
            dl.close()
    finally:
        if src is not None:
            src.close()
    summary = {"metric": f"GPU idle % vs step rate / feed rate ({a.family}, {a.source_dtype if a.family == 'images' else 'int32 tokens'})",
               "feed_per_s": round(feed, 1), "unit": unit, "batch": B, "points": len(points),
               "max_abs_error_pp": round(max(abs(p["error_pp"]) for p in points), 3) if points else None,
               "consumer_wait_s": round(stats.get("consumer_wait_s", 0.0), 3)}
    print(json.dumps(summary), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            for p in points:
                f.write(json.dumps(p) + "\n")
            f.write(json.dumps(summary) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
