#!/usr/bin/env python3
"""Headline benchmark: samples/s fed to the GPU + GPU idle %, synthetic 3x224x224 bf16.

Metric and config from BASELINE.json ("samples/sec fed to GPU + GPU idle%,
synthetic 3x224x224 bf16 at 1/2/4/8 ranks"). One process per GPU, each rank =
one consumer with its own producer worker processes:

  producers (host, pinned shm windows of synthetic bf16 images, refreshed every
  round) --hipMemcpyAsync on the prefetch stream--> HBM window ring
  --[global-shuffle all-to-all over RCCL when --exchange > 0]-->
  per-batch fused gfx950 Feistel-permutation gather --> bf16 [B,3,224,224]
  on the compute stream --> consumer step.

Launch: under torchrun (RANK/WORLD_SIZE set) every process is one rank. Without
a launcher, ``--gpus N`` > 1 makes this process spawn the N rank processes
itself (before anything touches the GPU) and exit with their status; a
WORLD_SIZE that disagrees with ``--gpus`` is an error, never a silent 1-rank run.

With N > 1 every window also goes through the global-shuffle exchange: half of
its rows are traded with all peers in one RCCL all-to-all over xGMI (BASELINE
config 3), on the DP group (one communicator and device order with the DDP
all-reduce of phase 2, ``ddl_amd/parallel/order.py``).

Phase 1 (the reported ``value``): the consumer step is a checksum kernel that
reads every delivered byte, so the number is the loader's feed rate. Every
sample crosses PCIe in every step (each window is re-copied H2D each visit;
no caching). W warmup steps, then EXACTLY K timed steps bracketed by
barrier + synchronize; max time over ranks. ``value`` is the SMALLER of
  * delivered: samples handed to the consumer in the timed region / time, and
  * landed: samples whose bytes crossed PCIe inside the timed region / time,
    on the GPU clock: the native stager times every window copy on the device
    (an event when its stream reaches the copy, its retire event), HIP timing
    events bracket the region on the idle compute stream, and each copy counts
    with the share of its [start, end] inside the region (pro rata, so the
    ~1.4 ms window granularity no longer quantises a 27 ms region),
so windows staged in HBM before t0 cannot inflate a short run. Both rates are
in the JSON line, with the H2D bytes and GB/s of the timed region and the
older whole-window count (copies enqueued AND retired inside the region).
Phase 2 (``gpu_idle_pct``): a fixed-cost bf16 train step (PatchMLP fwd+bwd+SGD)
consumes the batches; the compute stream's idle fraction is measured with HIP
events (idle = 1 - busy/wall). That step is ~4x slower than the feed, so phase 3
(``gpu_idle_pct_r090``, ``pressure``) repeats the measurement behind a calibrated
step whose capacity is 0.9x the phase-1 feed: the loader as the near-bottleneck.
``benchmarks/bench_idle_sweep.py`` sweeps that step across the whole ratio range.

The line proves its own layout (``dist``, ``ddl_amd/parallel/report.py``): the DP group's backend and
size, the RCCL version, each rank's device index, PCI bus ID and UUID, and a device-timed all-to-all of
``--a2a-probe-mb`` on the DP group per rank (its xGMI egress rate). An N > 1 run that is not RCCL over N
distinct GPUs exits 3 before measuring anything, unless it is labelled a rehearsal (``DDL_REHEARSAL=1``:
gloo ranks sharing one card, or CPU ranks); ``dist.rehearsal`` says which.

vs_baseline = value / (28,500 samples/s x N): BASELINE.md's reference
ceiling for this shape (P=3 host producers, f32, no H2D) scaled linearly.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

REF_SAMPLES_PER_S_PER_GPU = 28_500.0


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--window", type=int, default=256, help="samples per producer window")
    ap.add_argument("--producers", type=int, default=3)
    ap.add_argument("--slots", type=int, default=None,
                    help="windows per producer (default: the producer's preferred_slots: 1, or 2 with --refill full)")
    ap.add_argument("--depth", type=int, default=4,
                    help="HBM prefetch depth (windows; 4 x 77 MB of HBM; the library default): deep enough that the "
                         "copy engine restarts "
                         "without a gap after the barrier + synchronize that opens the timed region "
                         "(archive/profiles/r3_variance: 20-step spread 176.7-188.1k at depth 2-3, 187.5-188.1k at 4)")
    ap.add_argument("--source-dtype", default="bfloat16", choices=["bfloat16", "uint8", "float32"])
    ap.add_argument("--refill", default="stamp", choices=["stamp", "full"],
                    help="producer work per round: stamp = one element per sample; full = rewrite every byte of "
                         "the window (a row permutation of the pristine window, as the reference's producers "
                         "shuffle theirs every round) with --producer-threads native host threads each")
    ap.add_argument("--producer-threads", type=int, default=None,
                    help="host threads per producer for --refill full (default 8; 4 for the cheap refills)")
    ap.add_argument("--shuffle", default="device", choices=["device", "none"])
    ap.add_argument("--exchange", type=float, default=None,
                    help="global-shuffle fraction per window over RCCL (default 0.5 when N>1, as the reference "
                         "harness's fraction_exchange; 0 disables)")
    ap.add_argument("--exchange-method", default="alltoall")
    ap.add_argument("--idle-steps", type=int, default=-1, help="phase-2 steps (default: = --steps; 0 disables)")
    ap.add_argument("--pressure-ratio", type=float, default=0.9,
                    help="phase 3: GPU idle %% behind a calibrated step whose capacity is this multiple of the "
                         "phase-1 feed (the loader as the near-bottleneck); 0 disables")
    ap.add_argument("--model-dim", type=int, default=384)
    ap.add_argument("--model-depth", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--order", default="window+indexed", choices=["window", "window+indexed"],
                    help="window: the headline only (producer windows, per-window device shuffle); "
                         "window+indexed: also the world-size-invariant global order (EpochOrder), gathered by the "
                         "producer-free zero-copy kernel straight from a node-shared pinned bf16 source, reported "
                         "next to the headline in the JSON line ('indexed')")
    ap.add_argument("--index-samples", type=int, default=4096,
                    help="indexed order: samples in the node-shared synthetic source")
    ap.add_argument("--index-threads", type=int, default=8,
                    help="indexed order: host gather threads per producer (IndexedProducer host_threads)")
    ap.add_argument("--index-no-prefault", action="store_true",
                    help="indexed order: skip the one-word-per-page touch of the mapped source (A/B)")
    ap.add_argument("--zc-blocks", type=int, default=None,
                    help="indexed order, zero-copy path: workgroups of the PCIe gather (ZeroCopyLoader max_blocks; "
                         "default: its own choice, 32 for bf16)")
    ap.add_argument("--zc-handoff", default="host", choices=["host", "device"],
                    help="indexed order, zero-copy path: how a batch is handed to the consumer's stream")
    ap.add_argument("--dispatch", default="auto", choices=["auto", "inline", "lookahead", "python"],
                    help="per-batch dispatch: the native engine (auto / inline / lookahead) or the Python path")
    ap.add_argument("--a2a-probe-mb", type=float, default=32.0,
                    help="size of the device-timed all-to-all on the DP group that opens the run (the 'dist' block's "
                         "per-rank xGMI rate); 0 skips it")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--debug-log", action="store_true",
                    help="slow host iterations of the timed loop and long per-window stager waits in the JSON line")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int, argv: list[str]) -> int:
    """Run this script as ``n`` rank processes on this node (torchrun-style env); return their status.

    Called before anything touches the GPU. Rank 0's stdout is passed through (the JSON line);
    if any rank fails the others are terminated and the failure's exit code is returned.
    """
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        out = None if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env, stdout=out))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench: rank {procs.index(p)} exited with {code}; stopping the others", file=sys.stderr)
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


_T0 = time.perf_counter()


def _progress(env, what: str) -> None:
    """One line on stderr (rank 0) as each phase starts: a run of many phases is never silent for minutes."""
    if env.rank == 0:
        print(f"bench: {what} (+{time.perf_counter() - _T0:.1f} s)", file=sys.stderr, flush=True)


def phase2(args, env, dev, it, idle_steps: int, barrier, sync) -> dict:
    """GPU idle % behind a fixed-cost bf16 train step (DDP gradient all-reduce over RCCL when N > 1)."""
    _progress(env, "phase 2: idle behind the PatchMLP step")
    import torch
    import torch.distributed as dist

    from ddl_amd.models.trainstep import TrainStep
    from ddl_amd.utils.tracing import ComputeIdleMeter, trace_range

    step = TrainStep(dev, dim=args.model_dim, depth=args.model_depth,
                     process_group=env.process_group if env.world_size > 1 else None)
    for _ in range(args.warmup // 2):
        (x,) = next(it)
        step(x)
    meter = ComputeIdleMeter() if dev.type == "cuda" else None
    barrier()
    t2 = time.perf_counter()
    with trace_range("bench.phase2"):
        for _ in range(idle_steps):
            (x,) = next(it)
            if meter:
                meter.step_begin()
            step(x)
            if meter:
                meter.step_end()
        sync()
    t3 = time.perf_counter()
    idle = meter.result() if meter else {"gpu_idle_pct": float("nan"), "busy_ms": 0.0, "wall_ms": 0.0}
    idle["train_samples_per_s"] = args.batch * idle_steps * env.world_size / (t3 - t2)
    if env.world_size > 1:
        t = torch.tensor([idle["gpu_idle_pct"]], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
        idle["gpu_idle_pct"] = float(t.item())
    return idle


_FEED_DRAIN = 64  # batches: > HBM ring (depth 4 + 1) + producer slots + the indexed paths' prefetch


def pressure_phase(args, env, dev, it, feed_per_rank: float, barrier, sync, dl=None) -> dict:
    """GPU idle % with the LOADER as the near-bottleneck: a calibrated step (reads the whole batch, then a
    bf16 GEMM chain, ``CalibratedStep``) sized so its capacity is ``--pressure-ratio`` x this rank's phase-1
    feed, re-sized twice from its busy time measured in this very loop, then timed. Behind the PatchMLP
    step of phase 2 (~4x slower than the feed) any loader shows ~0 idle; here a loader that does not
    overlap its copies and kernels with the step shows up directly (``benchmarks/bench_idle_sweep.py``
    sweeps the whole ratio range)."""
    import torch
    import torch.distributed as dist

    from ddl_amd.models.trainstep import CalibratedStep
    from ddl_amd.utils.tracing import ComputeIdleMeter, trace_range

    from ddl_amd import ops

    _progress(env, "pressure phase: step at %.2fx the feed" % args.pressure_ratio)
    r, B = args.pressure_ratio, args.batch
    # the feed this phase runs against: re-measured here over >= 100 batches with the checksum consumer
    # (phase 1's region can be as short as 20 steps, and the loader's state after phase 2 -- copy streams,
    # ring -- is what the step will see); the step is sized from it, and its ratio is reported against it.
    # Phase 2's step is slower than the feed, so the loader enters this phase with every ring full: the first
    # batches come out of those rings at kernel speed, not at the feed rate, and a feed timed over them reads
    # ~4% high on the window path (198.7k vs 191.5k), sizing the step at an effective ratio of ~0.93 instead
    # of 0.9. _FEED_DRAIN untimed batches (more than the rings of every path hold) empty them first.
    acc = ops.ChecksumAccumulator(dev)
    for _ in range(_FEED_DRAIN):
        acc.add(next(it)[0])
    n_feed = max(args.steps, 100)
    sync()
    t0 = time.perf_counter()
    for _ in range(n_feed):
        acc.add(next(it)[0])  # the loaders' iterators here yield a tuple (the batch's column groups)
    sync()
    feed = B * n_feed / (time.perf_counter() - t0)
    step = CalibratedStep(dev, step_ms=1000.0 * B / (r * feed))
    step.calibrate(next(it)[0])
    for _ in range(max(2, args.warmup // 2)):
        step(next(it)[0])
    for _ in range(2):  # re-size from the busy time on the loader's batches (clocks, memory traffic)
        tm = ComputeIdleMeter()
        for _ in range(30):
            (x,) = next(it)
            tm.step_begin()
            step(x)
            tm.step_end()
        sync()
        tr = tm.result()
        step.tune(tr["busy_ms"] / max(1, tr["steps"]))
    n = max(args.steps, 300)
    stager = getattr(dl, "_stager", None)
    attempts = 0
    while True:
        # the timed loop; its busy time can land off target (the tune passes run while the loader refills its
        # ring after calibrate's synchronizations, so the GEMMs there see more interference than in steady
        # state): then re-size from THIS loop's busy time and time again, at most 3 times. Every rank makes
        # the same decision (MAX over ranks), so all of them fetch the same number of batches.
        attempts += 1
        _progress(env, f"pressure phase: timed loop {attempts} ({n} steps)")
        meter = ComputeIdleMeter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        t0 = time.perf_counter()
        e0.record()
        with trace_range("bench.pressure"):
            for _ in range(n):
                (x,) = next(it)
                meter.step_begin()
                step(x)
                meter.step_end()
            e1.record()
            sync()
        el = time.perf_counter() - t0
        res = meter.result()
        busy = res["busy_ms"] / max(1, res["steps"])
        cap = 1000.0 * B / busy
        retry = attempts < 3 and abs(cap / feed - r) > 0.03
        if env.world_size > 1:
            t = torch.tensor([1.0 if retry else 0.0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
            retry = bool(t.item() > 0)
        if not retry:
            break
        step.correct(busy)
    out = {"ratio_target": r, "ratio_measured": round(cap / feed, 3), "steps": n, "attempts": attempts,
           "feed_samples_per_s": round(feed, 1), "phase1_feed_samples_per_s": round(feed_per_rank, 1),
           "step_ms": round(busy, 4), "gpu_idle_pct": res["gpu_idle_pct"], "gaps_us": res.get("gaps_us"),
           "predicted_idle_pct": round(100.0 * max(0.0, 1.0 - feed / cap), 3),
           "achieved_samples_per_s": B * n * env.world_size / el}
    if stager is not None:  # how the window copies ran meanwhile (the auto policy's one-stream mode)
        out["copies"] = stager.copy_summary(e0, e1)
    if env.world_size > 1:
        t = torch.tensor([out["gpu_idle_pct"]], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
        out["gpu_idle_pct"] = float(t.item())
    out["gpu_idle_pct"] = round(out["gpu_idle_pct"], 3)
    out["achieved_samples_per_s"] = round(out["achieved_samples_per_s"], 1)
    return out


def _timed_feed(args, env, it, acc, barrier, sync, label: str, dl=None) -> tuple[float, float, dict]:
    """Warmup, then exactly ``args.steps`` checksum-consumed batches bracketed by barrier + synchronize;
    (samples/s over all ranks from the max elapsed time, ms per step, accounting). With ``dl`` (a loader that
    stages windows of ``args.batch`` samples through the H2D stager, copy timing on) the rate is the smaller of
    the delivered rate and the landed one -- the window bytes that crossed PCIe inside the region, on the device
    clock, pro rata -- as for the headline: windows staged before the region opened do not count."""
    import torch
    import torch.distributed as dist

    from ddl_amd.utils.tracing import trace_range

    _progress(env, f"feed: {label}")
    for _ in range(args.warmup):
        acc.add(next(it))
    stager = getattr(dl, "_stager", None) if dl is not None else None
    ev0 = ev1 = None
    if stager is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    if ev0 is not None:
        ev0.record()
    with trace_range(label):
        for _ in range(args.steps):
            acc.add(next(it))
        sync()
    el = time.perf_counter() - t0
    if ev1 is not None:
        ev1.record()
    landed = None
    if stager is not None:
        pro = stager.bytes_in_interval(ev0, ev1)
        landed = pro["windows"] * args.batch if pro.get("ok") else None
    barrier()
    t = torch.tensor([el, -1.0 if landed is None else landed], dtype=torch.float64)
    if env.world_size > 1:
        parts = [torch.empty_like(t) for _ in range(env.world_size)]
        dist.all_gather(parts, t, group=env.control_group)
    else:
        parts = [t]
    el = max(float(p[0]) for p in parts)
    delivered = args.batch * args.steps * env.world_size / el
    info = {"delivered_samples_per_s": round(delivered, 1)}
    rate = delivered
    if all(float(p[1]) >= 0 for p in parts):
        landed_rate = sum(float(p[1]) for p in parts) / el
        info["landed_samples_per_s"] = round(landed_rate, 1)
        rate = min(delivered, landed_rate)
    return rate, 1000 * el / args.steps, info


def _idle_behind_step(args, env, dev, it, barrier, sync) -> float | None:
    """GPU idle % behind the PatchMLP step (phase 2's measurement) on the batches of ``it``."""
    _progress(env, "idle behind the PatchMLP step")
    import torch
    import torch.distributed as dist

    from ddl_amd.models.trainstep import TrainStep
    from ddl_amd.utils.tracing import ComputeIdleMeter

    idle_steps = args.steps if args.idle_steps < 0 else args.idle_steps
    if not idle_steps or dev.type != "cuda":
        return None
    step = TrainStep(dev, dim=args.model_dim, depth=args.model_depth,
                     process_group=env.process_group if env.world_size > 1 else None)
    for _ in range(max(1, args.warmup // 2)):
        step(next(it))
    meter = ComputeIdleMeter()
    barrier()
    for _ in range(idle_steps):
        x = next(it)
        meter.step_begin()
        step(x)
        meter.step_end()
    sync()
    idle = meter.result()["gpu_idle_pct"]
    if env.world_size > 1:
        t = torch.tensor([idle], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
        idle = float(t.item())
    return round(idle, 3)


def indexed_phase(args, env, dev, barrier, sync, spare=None) -> dict:
    """The world-size-invariant order: every global batch is positions [g*GB, (g+1)*GB) of the epoch's
    Feistel permutation over a node-shared source, rank r taking its contiguous slice (the union over
    ranks is the same batch at any N). Two paths deliver it, each timed like the headline (checksum
    consumer, barrier + synchronize around exactly ``--steps`` batches), then GPU idle % behind the
    PatchMLP step:

    * ``value`` -- producers (``IndexedProducer`` on the spare producer set ``spare``, spawned with the
      headline's): each window is one local batch gathered on the host in the epoch order (native
      streaming-store gather) and staged like the headline's windows (direct DMA);
    * ``zero_copy`` -- ``ZeroCopyLoader``: a gfx950 kernel gathers the rank's slice straight from the
      pinned, device-mapped source over PCIe (no producers, no host copies; no host DRAM writes, which
      matters when four ranks share a socket).
    """
    import torch

    import ddl_amd
    from ddl_amd import ops
    from ddl_amd.models.datasets import numa_local_source
    from ddl_amd.models.producers import IndexedProducer
    from ddl_amd.zerocopy import ZeroCopyLoader

    shape = (3, 224, 224)
    n = max(args.index_samples, args.batch * env.world_size)
    name = f"ddl_amd_bench_idx_{os.environ.get('MASTER_PORT', os.getpid())}"

    def fill(t):  # every page written (resident on the replica's node); sample i's first element is i
        t.view(torch.uint8).fill_(0x3C)
        t.view(n, -1)[:, 0] = torch.arange(n, dtype=torch.float32).to(torch.bfloat16)

    def forever(dl):  # batches as one tensor (a window loader yields a tuple of column groups)
        while True:
            for b in dl:
                yield b[0] if isinstance(b, (tuple, list)) else b

    # one replica per NUMA node of the node's GPUs: no GPU gathers across the socket link
    src, node, _ = numa_local_source(name, n, shape, torch.bfloat16, env, fill=fill)
    out = {"order": "indexed (EpochOrder, world-size-invariant) from a NUMA-local bf16 replica of the "
                    "node-shared source", "source_samples": n}
    try:
        pages = src.page_nodes(64)
        out["numa"] = {"gpu_node": node, "source_pages_on_gpu_node_pct":
                       round(100.0 * sum(1 for p in pages if p == node) / max(1, len(pages)), 1)
                       if node is not None else None}
        acc = ops.ChecksumAccumulator(dev)
        idle_steps = args.steps if args.idle_steps < 0 else args.idle_steps
        if spare is not None:
            gb = args.batch * env.world_size
            bpe = n // gb
            total = args.warmup + args.steps + (max(1, args.warmup // 2) + idle_steps if idle_steps else 0) \
                + _pressure_batches(args)
            dl = ddl_amd.DistributedDataLoader(
                IndexedProducer(src, gb, seed=args.seed, host_threads=args.index_threads), args.batch, spare,
                math.ceil(total / bpe) + 2, env=env, device=dev, auto_mark=True,
                order=ddl_amd.OrderSpec(mode="indexed"),
                staging=ddl_amd.StagingSpec(n_slots=2, copy_timing=True),  # copy timing: the landed-bytes accounting
                output=ddl_amd.OutputSpec(copy_batches=False))  # views, as the headline's batches are: the checksum
            # reads them in stream order before the window's release (auto_mark would copy every batch, 77 MB D2D)
            it = forever(dl)
            w0 = dl.stats().get("stager_wait_producer_s", 0.0)
            rate, ms, acct = _timed_feed(args, env, it, acc, barrier, sync, "bench.indexed", dl=dl)
            st = dl.stats()
            out.update({"path": f"producers (IndexedProducer: host gather in the epoch order, 2 slots x "
                                f"{args.index_threads} threads, direct-DMA staging)",
                        "value": round(rate, 1), "ms_per_step": round(ms, 4), **acct,
                        "h2d_direct_dma": bool(st.get("direct_dma", False)),
                        # the stager's waits for producers over warmup + timed steps (diagnostic)
                        "stager_wait_producer_s": round(st.get("stager_wait_producer_s", 0.0) - w0, 4),
                        "producer_fill_us_per_round": [round(p["fill_ns_total"] / max(1, p["rounds"]) / 1e3, 1)
                                                       for p in st.get("producers", [])]})
            out["gpu_idle_pct"] = _idle_behind_step(args, env, dev, it, barrier, sync)
            out.update(_pressure_sub(args, env, dev, it, rate, barrier, sync, dl=dl))
            dl.close()
        zc = ZeroCopyLoader(src, args.batch * env.world_size, env, seed=args.seed, out_dtype=torch.bfloat16,
                            device=dev, prefault=not args.index_no_prefault, max_blocks=args.zc_blocks,
                            handoff=args.zc_handoff)
        it = forever(zc)
        rate, ms, _ = _timed_feed(args, env, it, acc, barrier, sync, "bench.indexed_zero_copy")
        zres = {"path": "zero-copy gfx950 gather over PCIe from the pinned, device-mapped source",
                "value": round(rate, 1), "ms_per_step": round(ms, 4), "prefault_s": zc.stats().get("prefault_s"),
                "max_blocks": zc.max_blocks, "handoff": zc.handoff}
        if spare is None:
            zres["gpu_idle_pct"] = _idle_behind_step(args, env, dev, it, barrier, sync)
        # the zero-copy gather holds CUs for its whole PCIe transfer: its idle behind a step at 0.9x the feed
        # is the number that compares it with the producer path
        zres.update(_pressure_sub(args, env, dev, it, rate, barrier, sync))
        if spare is None:
            out.update(zres)
        else:
            out["zero_copy"] = zres
        zc.close()
        return out
    finally:
        if env.world_size > 1:
            import torch.distributed as dist

            dist.barrier(group=env.control_group)  # every rank has unmapped its view before the unlink
        src.close()


def _pressure_batches(args) -> int:
    """Batches ``pressure_phase`` draws (an upper bound: calibration, tune passes, at most 3 timed loops)."""
    if args.pressure_ratio <= 0:
        return 0
    return _FEED_DRAIN + 1 + max(2, args.warmup // 2) + 60 + max(args.steps, 100) + 3 * max(args.steps, 300)


def _pressure_sub(args, env, dev, it, feed_total: float, barrier, sync, dl=None) -> dict:
    """Phase 3 on a sub-path's batches (``it`` yields tensors): ``gpu_idle_pct_r090`` + the pressure record."""
    if args.pressure_ratio <= 0 or dev.type != "cuda":
        return {}
    key = f"gpu_idle_pct_r{round(100 * args.pressure_ratio):03d}"
    try:
        pr = pressure_phase(args, env, dev, ((x,) for x in it), feed_total / env.world_size, barrier, sync, dl=dl)
    except Exception as e:  # the sub-path's feed rate is still reported
        import traceback

        traceback.print_exc()
        return {key: None, "pressure": {"error": repr(e)[:300]}}
    return {key: pr["gpu_idle_pct"], "pressure": pr}


def _landed(dl) -> tuple[int, int]:
    st = getattr(dl, "_stager", None)
    if st is None:  # CPU rehearsal: the host path has no H2D; every delivered window counts
        return dl.window, 0
    st.settle()  # called right after a device sync: count every copy that has completed, no retire lag
    return st.windows_landed, st.bytes_landed


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return self_launch(args.gpus, argv)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; refusing to run",
              file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd import Marker, ops
    from ddl_amd.models.producers import ImageWindowProducer
    from ddl_amd.parallel.order import LEDGER, check_same_order
    from ddl_amd.parallel.report import dist_block, require_verified
    from ddl_amd import _native
    from ddl_amd.utils.numa import gpu_numa_node
    from ddl_amd.utils.tracing import trace_range

    rt = _native.runtime()  # CLOCK_MONOTONIC now_ns(), the native stager's clock
    n_world = int(os.environ.get("WORLD_SIZE", "1"))
    LEDGER.enable(n_world > 1)  # record every collective at issue; digests compared across ranks at the end
    idle_steps = args.steps if args.idle_steps < 0 else args.idle_steps
    if args.exchange is None:
        args.exchange = 0.5 if n_world > 1 else 0.0
    total_steps = args.warmup + args.steps + (args.warmup // 2 + idle_steps if idle_steps else 0)
    total_steps += _pressure_batches(args)
    bpw = args.window // args.batch
    if bpw < 1:
        raise SystemExit("--window must hold at least one --batch")
    n_epochs = math.ceil(total_steps / bpw) + 1
    shape = (3, 224, 224)
    sample_bytes = math.prod(shape) * torch.empty((), dtype=getattr(torch, args.source_dtype)).element_size()

    # the indexed phase's producers are spawned with the headline's, before anything touches the GPU
    spares = 1 if args.order == "window+indexed" and args.producers > 0 else 0
    with ddl_amd.start(n_producers=args.producers, spare_connections=spares) as (env, conn):
        dev = torch.device(env.device)
        # the run proves its own layout: RCCL over N distinct GPUs (or a labelled rehearsal), with a
        # device-timed all-to-all on the DP group as the per-rank xGMI rate (parallel/report.py)
        dist_info = dist_block(env, int(args.a2a_probe_mb * (1 << 20)))
        refuse = require_verified(dist_info)
        if refuse is not None:
            print(f"bench: {refuse}; refusing to report an unverified dp{env.world_size} number", file=sys.stderr)
            if env.rank == 0:
                print("bench: dist = " + json.dumps({k: v for k, v in dist_info.items() if k != "ranks"}),
                      file=sys.stderr)
            return 3
        producer = ImageWindowProducer(args.window, shape, args.source_dtype, seed=args.seed, refill=args.refill,
                                       host_threads=args.producer_threads)
        norm = None
        if args.source_dtype == "uint8":
            norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225], "layout": "chw"}
        dl = ddl_amd.DistributedDataLoader(
            producer, args.batch, conn, n_epochs, args.exchange, args.exchange_method, env.rank, env.world_size,
            env=env, device=dev, output=ddl_amd.OutputSpec(dtype=torch.bfloat16, normalize=norm),
            order=ddl_amd.OrderSpec(shuffle=args.shuffle, seed=args.seed),
            staging=ddl_amd.StagingSpec(
                n_slots=args.slots, prefetch_depth=args.depth,
                native_dispatch=False if args.dispatch == "python" else args.dispatch,
                copy_timing=True))  # device times of every window copy: the pro-rata H2D accounting below
        acc = ops.ChecksumAccumulator(dev)  # one streaming launch per batch

        def batches():
            while True:
                for i in range(len(dl)):
                    yield dl[i]
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)

        it = batches()

        def sync():
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)

        def barrier():
            if env.world_size > 1:
                dist.barrier(group=env.control_group)
            sync()

        # ---------------- phase 1: feed rate
        _progress(env, f"phase 1: the headline feed over {args.steps} steps")
        for _ in range(args.warmup):
            (x,) = next(it)
            acc.add(x)
        prod0 = conn.producer_stats()  # diagnostics: read before the region opens
        wait_prod0 = dl.stats().get("stager_wait_producer_s", 0.0)
        host_log = args.debug_log
        ticks = []
        barrier()
        # the region's H2D work, on the GPU clock: events bracket the region on the (idle) compute stream, and
        # every window copy is timed on the device, so exactly the bytes that crossed PCIe inside the region
        # count (pro rata for the copies in flight at either end); the older whole-window counts (copies
        # ENQUEUED inside the region, native CLOCK_MONOTONIC timestamps) stay in the JSON as diagnostics
        ev0 = ev1 = None
        if dev.type == "cuda":
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        if ev0 is not None:
            ev0.record()
        t0_ns = rt.now_ns()
        w_land0, b_land0 = _landed(dl)
        w_cur0 = dl.window
        bytes_enq0 = dl._stager.bytes_h2d if dl._stager is not None else 0
        n_post0 = len(dl._stager.post_waits) if dl._stager is not None else 0
        with trace_range("bench.phase1"):  # roctx: lets tools/trace_idle.py find the timed region
            for _ in range(args.steps):
                (x,) = next(it)
                acc.add(x)
                if host_log:
                    ticks.append(time.perf_counter())
            sync()
        t1 = time.perf_counter()
        if ev1 is not None:
            ev1.record()
        t1_ns = rt.now_ns()
        # complete right now (before settle(): a copy still in flight at t1 must not finish into the count)
        cb = dl._stager._native.copies_between(t0_ns, t1_ns) if dl._stager is not None else None
        w_land1, b_land1 = _landed(dl)
        bytes_enq1 = dl._stager.bytes_h2d if dl._stager is not None else 0
        post_waits = dl._stager.post_waits[n_post0:] if dl._stager is not None else []
        # CPU rehearsal: the host path has no H2D; every delivered window counts
        n_in, b_in = cb[:2] if cb is not None else (w_land1 - w_land0, 0)
        cb_complete = bool(cb[2]) if cb is not None else None  # False: the copy log was trimmed in the region
        pro = dl._stager.bytes_in_interval(ev0, ev1) if dl._stager is not None and ev0 is not None else None
        if pro is not None and pro["ok"]:
            # the device interval is the region as the GPU saw it; its length next to the host's is a check
            n_in_prorata, b_in_prorata = pro["windows"], pro["bytes"]
        else:
            n_in_prorata, b_in_prorata = float(n_in), float(b_in)
        prod1 = conn.producer_stats()
        barrier()
        elapsed = t1 - t0
        landed_samples = n_in_prorata * args.window
        mine = {
            "rank": env.rank,
            "elapsed_s": elapsed,
            "delivered_per_s": args.batch * args.steps / elapsed,
            "landed_per_s": landed_samples / elapsed,
            "h2d_bytes_timed": int(b_in_prorata),
            "h2d_gbps_timed": b_in_prorata / elapsed / 1e9,
            "h2d_accounting": ("device-timed pro rata" if pro is not None and pro["ok"] else
                               "whole windows" if cb_complete is not False else "whole windows (INCOMPLETE log)"),
            "h2d_copy_log_complete": cb_complete,
            "device_region_ms": round(pro["t1_ms"] - pro["t0_ms"], 4) if pro is not None and pro["ok"] else None,
            "h2d_copies_overlapping_region": pro["copies"] if pro is not None else None,
            # device-timed link occupancy in the region: share of it with >= 1 / 2 window copies running
            "h2d_link_busy_pct": (round(100.0 * pro["busy_ms"] / max(1e-9, pro["t1_ms"] - pro["t0_ms"]), 2)
                                  if pro is not None and pro["ok"] else None),
            "h2d_two_copies_pct": (round(100.0 * pro["overlap_ms"] / max(1e-9, pro["t1_ms"] - pro["t0_ms"]), 2)
                                   if pro is not None and pro["ok"] else None),
            "h2d_copies_per_stream": list(pro["copies_per_stream"]) if pro is not None and pro["ok"] else None,
            # window copies straight onto SDMA engines through ROCr (True) or on HIP copy streams
            "h2d_direct_dma": bool(getattr(getattr(dl, "_stager", None), "direct_dma", False)),
            "h2d_bytes_whole_windows_enqueued_and_retired_in_region": b_in,
            "h2d_bytes_landed_any_enqueue_time": b_land1 - b_land0,
            "h2d_enqueued_bytes_timed": bytes_enq1 - bytes_enq0,
            "windows_prestaged_at_t0": max(0, w_land0 - w_cur0),
            "numa_node": gpu_numa_node(env.local_rank) if dev.type == "cuda" else None,
            "cpus": ({"consumer": len(conn.cpu_layout["consumer_cpus"]),
                      "consumer_reserved": len(conn.cpu_layout["consumer_reserved_cpus"]),
                      "producers": len(conn.cpu_layout["producer_cpus"])} if conn.cpu_layout
                     else {"shared": len(os.sched_getaffinity(0))}),
        }
        stats = dl.stats()
        if host_log:  # per-iteration host time of the timed loop (debug): the slow iterations
            dts = [b - a for a, b in zip([t0] + ticks[:-1], ticks)]
            mine["host_iter_ms_slow"] = [(i, round(1e3 * d, 2)) for i, d in enumerate(dts) if d > 0.002]
        if args.debug_log and dl._stager is not None:  # per-window producer waits (debug)
            mine["stager_step_log_us"] = [[e[0]] + [round(x / 1e3, 1) for x in e[1:6]]
                                          for e in dl._stager._native.wait_log if max(e[1:6]) > 500_000]
        # producer side of the timed region: rounds filled, fill rate while filling, busy fraction
        win_bytes = args.window * sample_bytes
        rounds = [b["rounds"] - a["rounds"] for a, b in zip(prod0, prod1)]
        fill_s = [(b["fill_ns_total"] - a["fill_ns_total"]) * 1e-9 for a, b in zip(prod0, prod1)]
        mine["producers"] = {
            "refill": args.refill,
            "rounds_timed": sum(rounds),
            "fill_gbps_per_producer": [round(r * win_bytes / s / 1e9, 2) if s > 0 else None
                                       for r, s in zip(rounds, fill_s)],
            "fill_busy_pct": [round(100.0 * s / elapsed, 1) for s in fill_s],
            "filled_gbps_total": round(sum(rounds) * win_bytes / elapsed / 1e9, 2),
        }
        mine["stager_wait_producer_s_timed"] = round(stats.get("stager_wait_producer_s", 0.0) - wait_prod0, 4)
        nd = stats.get("native_dispatch")
        mine["dispatch"] = {"mode": nd.get("mode"), "handoff": nd.get("handoff"),
                            "host_us_per_batch": nd.get("host_us_per_batch"),
                            "compute_waits": nd.get("compute_waits")} if nd else {"mode": "python"}
        mine["stager_wait_producer_s"] = round(stats.get("stager_wait_producer_s", 0.0), 4)
        mine["exchange_issue_wait_s"] = stats.get("exchange_issue_wait_s", 0.0)
        if post_waits:  # the timed region's per-window host waits at the exchange's issue point
            from ddl_amd.staging import issue_wait_summary

            mine["exchange_issue_wait_timed"] = issue_wait_summary(post_waits)
        mine["consumer_wait_s"] = round(stats["consumer_wait_s"], 4)
        ex = getattr(dl, "_exchange_fn", None)
        if ex is not None:
            mine.update(ex.stats())
        per_rank = [mine]
        if env.world_size > 1:
            per_rank = [None] * env.world_size
            dist.all_gather_object(per_rank, mine, group=env.control_group)
        elapsed = max(r["elapsed_s"] for r in per_rank)
        delivered = args.batch * args.steps * env.world_size / elapsed
        landed = sum(r["landed_per_s"] * r["elapsed_s"] for r in per_rank) / elapsed
        value = min(delivered, landed) if landed > 0 else delivered

        # ---------------- phase 2: GPU idle % behind a fixed-cost train step
        idle = {}
        phase2_error = None
        try:
            if idle_steps:
                idle = phase2(args, env, dev, it, idle_steps, barrier, sync)
        except Exception as e:  # the feed rate (phase 1) is still reported; the error goes into the JSON line
            import traceback

            traceback.print_exc()
            phase2_error, idle = repr(e)[:300], {}
        # ---------------- phase 3: GPU idle % with the loader as the near-bottleneck
        pressure = None
        if args.pressure_ratio > 0 and dev.type == "cuda":
            try:
                pressure = pressure_phase(args, env, dev, it, value / env.world_size, barrier, sync, dl=dl)
            except Exception as e:  # the headline is still reported
                import traceback

                traceback.print_exc()
                pressure = {"error": repr(e)[:300]}
        dl.close()
        order = check_same_order(env.control_group) if env.world_size > 1 else None
        indexed = None
        if args.order == "window+indexed":
            try:
                indexed = indexed_phase(args, env, dev, barrier, sync,
                                        spare=conn.spares[0] if conn is not None and conn.spares else None)
            except Exception as e:  # the headline is still reported
                import traceback

                traceback.print_exc()
                indexed = {"error": repr(e)[:300]}

        if env.rank == 0:
            for r in per_rank:
                for k in ("elapsed_s", "delivered_per_s", "landed_per_s", "h2d_gbps_timed"):
                    r[k] = round(r[k], 4 if k != "delivered_per_s" and k != "landed_per_s" else 1)
            out = {
                "metric": "samples/sec fed to GPU (synthetic 3x224x224 bf16)",
                "value": round(value, 1),
                "unit": "samples/s",
                "n_gpus": env.world_size,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": round(value / (REF_SAMPLES_PER_S_PER_GPU * env.world_size), 3),
                "dtype": "bf16",
                "data": f"synthetic (random {args.source_dtype} images, refreshed every producer round: "
                        f"{args.refill})",
                "config": {
                    "model": "ddl_amd loader: ImageNet-shape 3x224x224 bf16, pinned H2D prefetch stream",
                    "global_batch": args.batch * env.world_size,
                    "seq_len": None,
                    "parallelism": f"dp{env.world_size}",
                    "producers_per_gpu": args.producers,
                    "window_samples": args.window,
                    "prefetch_depth": args.depth,
                    "shuffle": args.shuffle,
                    "exchange_fraction": args.exchange,
                    "exchange_method": args.exchange_method if args.exchange > 0 else None,
                    "source_dtype": args.source_dtype,
                    "producer_refill": args.refill,
                    "producer_slots": dl.n_slots,
                    "producer_threads": producer.host_threads,
                    "dispatch": per_rank[0].get("dispatch", {}).get("mode"),
                },
                "delivered_samples_per_s": round(delivered, 1),
                "landed_samples_per_s": round(landed, 1),
                "h2d_bytes_timed": sum(r["h2d_bytes_timed"] for r in per_rank),
                "h2d_gbps_timed": round(sum(r["h2d_bytes_timed"] for r in per_rank) / elapsed / 1e9, 3),
                "sample_bytes": sample_bytes,
                "windows_prestaged_at_t0": max(r["windows_prestaged_at_t0"] for r in per_rank),
                "gpu_idle_pct": (None if not idle or math.isnan(idle["gpu_idle_pct"])
                                 else round(idle["gpu_idle_pct"], 3)),
                "train_step": None if not idle else {
                    "model": f"PatchMLP dim={args.model_dim} depth={args.model_depth} fwd+bwd+SGD bf16"
                             + (" (DDP all-reduce)" if env.world_size > 1 else ""),
                    "samples_per_s": round(idle["train_samples_per_s"], 1),
                    "busy_ms": round(idle["busy_ms"], 3), "wall_ms": round(idle["wall_ms"], 3)},
                "phase2_error": phase2_error,
                # the loader as the near-bottleneck: a calibrated step at --pressure-ratio x the feed
                f"gpu_idle_pct_r{round(100 * args.pressure_ratio):03d}": (pressure or {}).get("gpu_idle_pct"),
                "pressure": pressure,
                "collective_order": order,
                "dist": dist_info,
                "indexed": indexed,
                "per_rank": per_rank,
            }
            line = json.dumps(out)
            print(line, flush=True)
            if args.json_out:
                with open(args.json_out, "w") as f:
                    f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
