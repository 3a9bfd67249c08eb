#!/usr/bin/env python3
"""BASELINE config 4: token sequences, seq_len=4096, ragged H2D + on-device pad/pack collate.

Synthetic corpus (random token ids, lengths uniform in [min_len, 4096]) in node
shm; producers gather sequences in the world-size-invariant global order into
pinned windows (ragged: only real tokens cross PCIe); the consumer expands
them with the gfx950 pad_pack_tokens kernel. Reports tokens/s fed to the GPU
(real tokens, padding excluded) and batches/s. torchrun-compatible.
"""

import argparse
import json
import os
import sys
import time

import numpy as np


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64, help="sequences per rank per step")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--min-len", type=int, default=256)
    ap.add_argument("--n-seqs", type=int, default=8192)
    ap.add_argument("--producers", type=int, default=6)
    ap.add_argument("--slots", type=int, default=2, help="windows per producer (a producer fills one while the "
                                                          "previous is in flight)")
    ap.add_argument("--batches-per-window", type=int, default=8,
                    help="global batches per producer window (per-window costs amortised over k batches)")
    ap.add_argument("--host-threads", type=int, default=4, help="gather threads per producer")
    ap.add_argument("--token-rows", default="exact", choices=["exact", "fixed"],
                    help="pack mode: exact packed rows per batch, or the window layout's fixed max rows (padding)")
    ap.add_argument("--dispatch", default="auto", choices=["auto", "inline", "lookahead", "window", "python"])
    ap.add_argument("--mode", default="pack", choices=["pad", "pack"])
    ap.add_argument("--pack-order", default="ffd", choices=["in_order", "ffd"],
                    help="pack mode: first-fit-decreasing rows (measured 93%% dense) or in-order (~75%%)")
    ap.add_argument("--idle-steps", type=int, default=200,
                    help="phase 2: steps of a fixed-cost token train step, for GPU idle %% (0 disables)")
    ap.add_argument("--model-dim", type=int, default=256)
    ap.add_argument("--model-depth", type=int, default=2)
    ap.add_argument("--token-dtype", default="auto", choices=["auto", "int32", "uint16"],
                    help="token ids in the corpus and on the wire: auto = uint16 when every id is < 65536 (the "
                         "synthetic GPT-2-sized vocabulary is), else int32; uint16 ships 2 B per token over PCIe "
                         "and the pack kernel widens it to int32 input_ids (archive/profiles/r3_tok16)")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd import ops
    from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    name = f"ddl_amd_benchtok_{os.environ.get('MASTER_PORT', '0')}"
    src = None
    if int(os.environ.get("LOCAL_RANK", "0")) == 0:
        from ddl_amd.utils.numa import gpu_numa_node

        src = SharedTokenSource.synthetic(name, a.n_seqs, a.min_len, a.seq_len, seed=1, token_dtype=a.token_dtype)
        src.bind_to_node(gpu_numa_node(int(os.environ.get("LOCAL_RANK", "0"))))  # the producers' node
        from ddl_amd.models.datasets import SharedArraySource

        tb_seg = SharedArraySource(name + "_tb", 1, (1,), "int64", create=True)  # the wire dtype, for the node's ranks
        tb_seg.tensor().view(-1)[0] = src.token_bytes
    gb = a.batch * world
    try:
        with ddl_amd.start(n_producers=a.producers) as (env, conn):
            if env.world_size > 1:
                dist.barrier(group=env.control_group)
            if src is None:
                from ddl_amd.models.datasets import SharedArraySource

                # local rank 0 created the corpus; its wire dtype travels in the offsets segment's neighbour
                tb_view = SharedArraySource(name + "_tb", 1, (1,), "int64")  # held: its tensor maps the segment
                tb = int(tb_view.tensor().view(-1)[0])
                del tb_view
                t = SharedArraySource(name + "_tok", 0, (1,), torch.int32 if tb == 4 else torch.int16)
                o = SharedArraySource(name + "_off", a.n_seqs + 1, (1,), "int64")
                offs = o.tensor().view(-1).numpy()
                t.n = int(offs[-1])
                source = SharedTokenSource(t, o, int(np.diff(offs).max()))
            else:
                source = src
            n_epochs = (a.warmup + a.steps + a.idle_steps + a.warmup // 2) // (a.n_seqs // gb) + 2
            producer = TokenBatchProducer(source, gb, a.seq_len, a.mode,
                                          pack_order=a.pack_order if a.mode == "pack" else "in_order",
                                          batches_per_window=a.batches_per_window, host_threads=a.host_threads)
            dispatch = False if a.dispatch == "python" else a.dispatch
            dl = ddl_amd.DistributedDataLoader(producer, a.batch, conn, n_epochs, env=env, auto_mark=True,
                                               output=ddl_amd.OutputSpec(collate="tokens", token_rows=a.token_rows),
                                               staging=ddl_amd.StagingSpec(n_slots=a.slots,
                                                                           native_dispatch=dispatch),
                                               order=ddl_amd.OrderSpec(mode="indexed"))
            dev = torch.device(env.device)
            acc = ops.ChecksumAccumulator(dev)  # one streaming launch per batch

            def sync():  # the CPU rehearsal (DDL_DEVICE=cpu) has nothing to synchronise
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)

            def gen():
                while True:
                    yield from dl

            it = gen()
            real = 0
            for _ in range(a.warmup):
                b = next(it)
                acc.add(b["input_ids"])
            sync()
            if env.world_size > 1:
                dist.barrier(group=env.control_group)
            t0 = time.perf_counter()
            rows = 0
            for _ in range(a.steps):
                b = next(it)
                acc.add(b["input_ids"])
                rows += b.get("n_rows", b["input_ids"].shape[0])
                real += b["n_tokens"]  # counted from the delivered batches (producer tag), not estimated
            sync()
            dt = time.perf_counter() - t0
            st = dl.stats()
            if env.world_size > 1:
                t = torch.tensor([dt], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
                dt = float(t.item())
            idle = None
            if a.idle_steps and dev.type == "cuda":
                # phase 2: GPU idle % behind a fixed-cost bf16 token train step (BASELINE config 4)
                from ddl_amd.models.trainstep import TokenTrainStep
                from ddl_amd.utils.tracing import ComputeIdleMeter

                step = TokenTrainStep(dev, seq_len=a.seq_len, dim=a.model_dim, depth=a.model_depth)
                for _ in range(max(1, a.warmup // 2)):
                    step(next(it))
                meter = ComputeIdleMeter()
                sync()
                t2 = time.perf_counter()
                for _ in range(a.idle_steps):
                    b = next(it)
                    meter.step_begin()
                    step(b)
                    meter.step_end()
                sync()
                t3 = time.perf_counter()
                idle = meter.result()
                idle["train_sequences_per_s"] = a.idle_steps * a.batch * env.world_size / (t3 - t2)
                if env.world_size > 1:
                    t = torch.tensor([idle["gpu_idle_pct"]], dtype=torch.float64)
                    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.control_group)
                    idle["gpu_idle_pct"] = float(t.item())
            toks = source.offsets.tensor().view(-1).numpy()
            mean_len = float(np.diff(toks).mean())
            est_tokens = a.steps * a.batch * mean_len * env.world_size
            real_tokens = real
            if env.world_size > 1:
                t = torch.tensor([real], dtype=torch.float64)
                dist.all_reduce(t, group=env.control_group)
                real_tokens = float(t.item())
            dl.close()
            if env.rank == 0:
                print(json.dumps({
                    "metric": "tokens/s fed to GPU (seq_len 4096, on-device pad/pack)", "mode": a.mode,
                    "value": round(real_tokens / dt, 1), "unit": "tokens/s (real tokens delivered)",
                    "value_est_from_mean_len": round(est_tokens / dt, 1),
                    "sequences_per_s": round(a.steps * a.batch * env.world_size / dt, 1),
                    "packed_rows_per_step": round(rows / a.steps, 2),
                    "pack_order": a.pack_order if a.mode == "pack" else None,
                    "row_density": round(real / max(rows * a.seq_len, 1), 3),
                    "row_density_est": round(a.batch * mean_len / (rows / a.steps) / a.seq_len, 3),
                    "n_gpus": env.world_size,
                    "steps": a.steps, "ms_per_step": round(1000 * dt / a.steps, 3), "batch_seqs": a.batch,
                    "producers": a.producers, "host_threads": a.host_threads, "slots": a.slots,
                    "batches_per_window": dl.batches_per_window[0], "dispatch": a.dispatch,
                    "dispatch_mode": (st.get("native_dispatch") or {}).get("mode"), "token_rows": a.token_rows,
                    "mean_len": round(mean_len, 1),
                    "token_wire_dtype": "uint16" if source.token_bytes == 2 else "int32",
                    "h2d_token_gbps": round(real_tokens * source.token_bytes / dt / 1e9, 2),
                    "consumer_wait_s": round(st["consumer_wait_s"], 3),
                    "stager_wait_producer_s": round(st.get("stager_wait_producer_s", 0.0), 3),
                    # per producer: rounds, mean fill and mean slot-wait per round (us) -- where the feed goes
                    "producers_rounds_fill_wait_us": [
                        (p["rounds"], round(p["fill_ns_total"] / max(1, p["rounds"]) / 1e3, 1),
                         round(p["wait_ns_total"] / max(1, p["rounds"]) / 1e3, 1)) for p in st.get("producers", [])],
                    "gpu_idle_pct": None if idle is None else round(idle["gpu_idle_pct"], 3),
                    "train_step": None if idle is None else {
                        "model": f"TokenMLP dim={a.model_dim} depth={a.model_depth} fwd+bwd+SGD bf16",
                        "sequences_per_s": round(idle["train_sequences_per_s"], 1),
                        "busy_ms": round(idle["busy_ms"], 3), "wall_ms": round(idle["wall_ms"], 3)}}),
                    flush=True)
    finally:
        if src is not None:
            src.close()
            tb_seg.close()


if __name__ == "__main__":
    sys.exit(main())
