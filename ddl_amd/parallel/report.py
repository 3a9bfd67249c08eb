"""Self-verifying description of a multi-rank run: which backend, which GPUs, what xGMI rate.

The reference builds its topology from ``mpirun`` ranks and only checks that a GPU's ranks share a node
and that the rank count divides (reference ddl/ddl_env.py:12-30,58-81); nothing in its output says which
transport or which devices a run actually used. A benchmark line that claims ``dp8`` must prove it by
itself, so :func:`dist_block` gathers, over the gloo control group:

* the DP group's backend (RCCL is ``"nccl"`` on ROCm), its size and the RCCL version torch is linked with;
* per rank: host, local rank, device index, PCI bus ID and UUID of its GPU;
* per rank: a device-timed all-to-all of ``probe_bytes`` on the DP group (:func:`alltoall_probe`), i.e.
  the xGMI rate this rank's exchange traffic can get;

and sets ``verified`` only when the group is RCCL over ``world_size`` distinct GPUs (distinct PCI bus IDs on
every host). :func:`require_verified` turns an unverified N > 1 run into an error unless it is labelled a
rehearsal (``DDL_REHEARSAL=1``: gloo ranks sharing one card, or ranks on the CPU).
"""

from __future__ import annotations

import statistics
import time

from ..types import DDLEnv
from .env import device_identity, rehearsal
from .order import issue


def rccl_version() -> str | None:
    """The RCCL (``torch.cuda.nccl``) version torch is linked with, as ``"major.minor.patch"``."""
    try:
        import torch

        v = torch.cuda.nccl.version()
    except Exception:  # pragma: no cover - torch without RCCL
        return None
    return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)


def alltoall_probe(env: DDLEnv, probe_bytes: int = 32 << 20, iters: int = 8, warmup: int = 2) -> dict:
    """Time ``all_to_all_single`` of ``probe_bytes`` per rank on the DP group (a collective: every rank calls
    it at the same point). On a GPU each iteration is bracketed by HIP events on the current stream (the
    RCCL stream is ordered behind and before it by ProcessGroupNCCL), so the time is device time.

    ``out_gbps`` counts the bytes that leave the rank (``(W-1)/W`` of the buffer; the own chunk is a local
    copy), which is the per-GPU xGMI egress an all-to-all exchange drives; ``alg_gbps`` counts the whole
    buffer. Median and best over ``iters``."""
    import torch
    import torch.distributed as dist

    group = env.process_group
    if group is None:
        return {"skipped": "no process group"}
    W = dist.get_world_size(group)
    n = max(W, (int(probe_bytes) // (W * 16)) * W * 16)
    gpu = str(env.device).startswith("cuda")
    dev = torch.device(env.device if gpu else "cpu")
    send = torch.full((n,), env.rank & 0xFF, dtype=torch.uint8, device=dev)
    recv = torch.empty_like(send)
    times = []
    for i in range(warmup + iters):
        issue(env, group, "bench.alltoall_probe", i)
        if gpu:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dist.all_to_all_single(recv, send, group=group)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
        else:
            t0 = time.perf_counter()
            dist.all_to_all_single(recv, send, group=group)
            ms = 1e3 * (time.perf_counter() - t0)
        if i >= warmup:
            times.append(ms)
    chunk = n // W
    ok = all(int(recv[p * chunk]) == (p & 0xFF) for p in range(W))  # every peer's chunk landed in its place
    med, best = statistics.median(times), min(times)
    out_bytes = n * (W - 1) // W
    return {"bytes": n, "iters": iters, "ms_median": round(med, 4), "ms_best": round(best, 4),
            "out_gbps": round(out_bytes / med / 1e6, 2), "out_gbps_best": round(out_bytes / best / 1e6, 2),
            "alg_gbps": round(n / med / 1e6, 2), "device_timed": gpu, "data_ok": ok}


def dist_block(env: DDLEnv, probe_bytes: int = 32 << 20) -> dict:
    """The run's distributed identity (module doc). Collective at N > 1: call it on every rank."""
    import torch.distributed as dist

    mine = {"rank": env.rank, "host": env.hostname, "local_rank": env.local_rank, "device": env.device,
            **device_identity(env.device)}
    if env.process_group is not None and probe_bytes > 0:
        mine["alltoall"] = alltoall_probe(env, probe_bytes)
    ranks = [mine]
    if env.world_size > 1 and env.control_group is not None:
        ranks = [None] * env.world_size
        dist.all_gather_object(ranks, mine, group=env.control_group)
    backend = dist.get_backend(env.process_group) if env.process_group is not None else None
    group_size = dist.get_world_size(env.process_group) if env.process_group is not None else 1
    keys = [(r["host"], r.get("pci_bus_id") or r.get("uuid")) for r in ranks]
    gpus = [k for k in keys if k[1]]
    distinct = len(set(gpus))
    problems = []
    if env.world_size > 1:
        if backend != "nccl":
            problems.append(f"DP backend is {backend!r}, not RCCL ('nccl')")
        if group_size != env.world_size:
            problems.append(f"DP group has {group_size} ranks, the job {env.world_size}")
        if len(gpus) != env.world_size:
            problems.append(f"{env.world_size - len(gpus)} rank(s) are not on a GPU")
        elif distinct != env.world_size:
            problems.append(f"{env.world_size} ranks on {distinct} distinct GPU(s)")
        bad = [r["rank"] for r in ranks if r.get("alltoall", {}).get("data_ok") is False]
        if bad:
            problems.append(f"all-to-all probe delivered wrong bytes on ranks {bad}")
    a2a = [r["alltoall"]["out_gbps"] for r in ranks if "out_gbps" in r.get("alltoall", {})]
    return {
        "backend": backend,
        "group_size": group_size,
        "world_size": env.world_size,
        "rccl_version": rccl_version(),
        "distinct_gpus": distinct,
        "hosts": len({r["host"] for r in ranks}),
        "alltoall_out_gbps_min": min(a2a) if a2a else None,
        "verified": (not problems) if env.world_size > 1 else None,  # None: a single rank has nothing to verify
        "rehearsal": rehearsal(),
        "problems": problems,
        "ranks": ranks,
    }


def require_verified(block: dict) -> str | None:
    """An error message when an N > 1 run is not RCCL over N distinct GPUs and not labelled a rehearsal
    (``DDL_REHEARSAL=1``); None when the run may proceed."""
    if block["world_size"] <= 1 or block["verified"] or block["rehearsal"]:
        return None
    return ("multi-rank run is not RCCL over distinct GPUs: " + "; ".join(block["problems"])
            + " (set DDL_REHEARSAL=1 to run it as a labelled rehearsal)")
