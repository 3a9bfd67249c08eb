#!/usr/bin/env python3
"""BASELINE config 5: HBM-resident sharded dataset, exact global shuffle, prefetch-depth sweep.

A synthetic 3x224x224 dataset (bf16, or uint8 with on-device normalise) is
sharded across the ranks and loaded into HBM once; every step assembles a
batch of the world-size-invariant global permutation (gfx950 gather kernels +
RCCL all-to-all over xGMI for W > 1). Sweeps the prefetch depth; reports
samples/s fed (checksum consumer) per depth. torchrun-compatible.

``--replicate`` picks the layout at W > 1 (``ResidentGlobalLoader(replicate=)``): replicated (default when the
dataset fits in HBM: an all-gather over xGMI at bring-up, then no per-step collective) or sharded (a per-step
RCCL all-to-all of (W-1)/W of every batch).
"""

import argparse
import json
import os
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256, help="per-rank batch")
    ap.add_argument("--n-samples", type=int, default=16384, help="global dataset size")
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "uint8"])
    ap.add_argument("--depths", default="1,2,4")
    ap.add_argument("--replicate", default="auto", choices=["auto", "true", "false"],
                    help="replicated: every rank holds the whole dataset (1/W loaded from host per rank, the rest "
                         "all-gathered over xGMI once; no per-step collective); sharded: rank r holds rows "
                         "[r*S, (r+1)*S) and every step all-to-alls (W-1)/W of its batch; auto: replicated when "
                         "it fits in 80%% of free HBM")
    ap.add_argument("--idle-step-ms", type=float, default=0.0,
                    help="after the sweep: GPU idle %% behind a fixed-cost step of this many ms (a batch read + bf16 "
                         "GEMMs) fed by the loader at --depths' first depth, for each --handoff; 0 skips it")
    ap.add_argument("--handoffs", default="device",
                    help="comma list of hand-offs for the idle phase (device: the step's stream waits for the "
                         "batch's event; host: the host does)")
    ap.add_argument("--augment", action="store_true",
                    help="RandomResizedCrop(224) + flip + normalise on the device instead of the plain gather")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd import ops
    from ddl_amd.models.datasets import SharedArraySource
    from ddl_amd.parallel.report import dist_block, require_verified
    from ddl_amd.resident import ResidentGlobalLoader

    shape = (3, 224, 224)
    name = f"ddl_amd_benchres_{os.environ.get('MASTER_PORT', '0')}"
    creator = int(os.environ.get("LOCAL_RANK", "0")) == 0
    dt = torch.uint8 if a.dtype == "uint8" else torch.bfloat16
    src = SharedArraySource(name, a.n_samples, shape, dt, create=creator)
    results = []
    try:
        with ddl_amd.start(n_producers=0) as (env, _):
            if creator:
                # deterministic fill, sample i = (7 i + column) mod 251 (valid bf16 values); periodic in i with
                # period 251, so one block of 16 periods is built once and copied (multi-threaded) over the
                # whole array: an ImageNet-size (1.28M-sample, 193 GB uint8) source fills in seconds
                t = src.tensor().view(a.n_samples, -1)
                blk = min(251 * 16, a.n_samples)
                base = ((torch.arange(blk).view(-1, 1) * 7 + torch.arange(t.shape[1]).view(1, -1)) % 251).to(dt)
                for i in range(0, a.n_samples, blk):
                    n = min(blk, a.n_samples - i)
                    t[i:i + n].copy_(base[:n])
                del base
            if env.world_size > 1:
                dist.barrier(group=env.control_group)
            dist_info = dist_block(env, 32 << 20)  # backend, GPUs, per-rank all-to-all rate (parallel/report.py)
            refuse = require_verified(dist_info)
            if refuse is not None:
                print(f"bench_resident: {refuse}", file=sys.stderr)
                return 3
            norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225]} if a.dtype == "uint8" else None
            dev = torch.device(env.device)

            def sync():
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)
            for depth in [int(x) for x in a.depths.split(",")]:
                rep = {"auto": "auto", "true": True, "false": False}[a.replicate]
                dl = ResidentGlobalLoader(src, a.batch * env.world_size, env, seed=1, depth=depth,
                                          out_dtype=torch.bfloat16, normalize=norm, replicate=rep,
                                          augment={"size": (224, 224)} if a.augment else None)
                acc = ops.ChecksumAccumulator(dev)  # one streaming launch per batch

                def gen():
                    while True:
                        yield from dl

                it = gen()
                for _ in range(a.warmup):
                    acc.add(next(it))
                sync()
                if env.world_size > 1:
                    dist.barrier(group=env.control_group)
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    acc.add(next(it))
                sync()
                el = time.perf_counter() - t0
                if env.world_size > 1:
                    tt = torch.tensor([el], dtype=torch.float64)
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=env.control_group)
                    el = float(tt.item())
                st = dl.stats()
                dl.close()  # frees the shard; `it` still references dl
                results.append({"depth": depth, "samples_per_s": round(a.batch * a.steps * env.world_size / el, 1),
                                "ms_per_step": round(1000 * el / a.steps, 4),
                                "mode": "replicated" if st["replicated"] else "sharded",
                                # bring-up: host -> HBM of this rank's rows, then (replicated) the all-gather
                                "load_s": round(st["load_s"], 2), "replicate_s": round(st["replicate_s"], 2),
                                "resident_GB": round(st["shard_bytes"] / 1e9, 2),
                                "xgmi_GB_sent_per_rank_steps": round(st["bytes_exchanged"] / 1e9, 3),
                                "xgmi_GB_sent_per_rank_bringup": round(st["bytes_replicated"] / 1e9, 3)})
                del dl, it, acc
                if dev.type == "cuda":
                    torch.cuda.empty_cache()  # hand the freed shard back before the next depth allocates its own
            idle = []
            if a.idle_step_ms > 0 and dev.type == "cuda":
                from ddl_amd.models.trainstep import CalibratedStep
                from ddl_amd.utils.tracing import ComputeIdleMeter

                step = CalibratedStep(dev, step_ms=a.idle_step_ms)
                for handoff in a.handoffs.split(","):
                    dl = ResidentGlobalLoader(src, a.batch * env.world_size, env, seed=1,
                                              depth=int(a.depths.split(",")[0]), out_dtype=torch.bfloat16,
                                              normalize=norm, replicate={"auto": "auto", "true": True,
                                                                         "false": False}[a.replicate],
                                              handoff=handoff)

                    def gen2():
                        while True:
                            yield from dl

                    it2 = gen2()
                    step.calibrate(next(it2))  # size the GEMM chain to step_ms on this GPU (once per loader)
                    for _ in range(a.warmup):
                        step(next(it2))
                    sync()
                    meter = ComputeIdleMeter()
                    for _ in range(a.steps):
                        x = next(it2)
                        meter.step_begin()
                        step(x)
                        meter.step_end()
                    sync()
                    res = meter.result()
                    idle.append({"handoff": handoff, "step_ms": a.idle_step_ms,
                                 "busy_ms_per_step": round(res["busy_ms"] / max(1, res["steps"]), 4),
                                 "gpu_idle_pct": res["gpu_idle_pct"],
                                 "gaps_us": res.get("gaps_us"), "host_waits": dl.host_waits})
                    dl.close()
                    del dl, it2
            if env.rank == 0:
                print(json.dumps({"metric": "samples/s fed to GPU, HBM-resident exact global shuffle",
                                  "idle_behind_step": idle,
                                  "dist": dist_info,
                                  "augment": "RandomResizedCrop(224)+flip+normalise" if a.augment else None,
                                  "n_gpus": env.world_size, "batch_per_gpu": a.batch, "dtype_src": a.dtype,
                                  "dtype_out": "bf16", "n_samples": a.n_samples, "sweep": results}), flush=True)
    finally:
        src.close()


if __name__ == "__main__":
    sys.exit(main())
