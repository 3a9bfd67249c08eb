#!/usr/bin/env python3
"""Packed (or padded) token batches for LLM training, seq_len 4096 (BASELINE config 4).

    python examples/tokens_packed.py [--mode pad]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/tokens_packed.py

A tokenised corpus (flat int32 tokens + int64 sequence offsets) sits in node-shared
memory (``SharedTokenSource``; ``.create(name, tokens, offsets)`` for your own data).
Producers gather each step's sequences in the world-size-invariant global order
and ship them RAGGED, so only real tokens cross PCIe. The consumer expands a
batch on the GPU with the pad/pack kernel:

* ``pack``: sequences packed into rows of ``seq_len`` by first-fit decreasing
  (``pack_order="ffd"``, ~93% dense measured; long ones split).
  Returns ``input_ids``, ``attention_mask``, ``position_ids`` (restarting per
  sequence), ``segment_ids``, int32 ``cu_seqlens`` over ``input_ids[attention_mask.bool()]`` and
  ``max_seqlen`` (the varlen-attention inputs; one entry per segment).
* ``pad``: one sequence per row, padded with ``pad_id``.

``batches_per_window=k`` ships k consecutive global batches per producer window
(one producer round, one H2D copy and one stager hand-off per k batches).

``state_dict()`` is the indexed-kind cursor (seed, epoch, global batch), so a
job can resume at another world size.
"""

import argparse
import os

import torch

import ddl_amd
from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="pack", choices=["pack", "pad"])
    ap.add_argument("--n-seqs", type=int, default=1024)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--global-batch", type=int, default=32, help="sequences per global step")
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batches-per-window", type=int, default=4)
    a = ap.parse_args()

    name = f"ddl_amd_example_tok_{os.environ.get('MASTER_PORT', os.getpid())}"
    creator = int(os.environ.get("LOCAL_RANK", "0")) == 0
    src = SharedTokenSource.synthetic(name, a.n_seqs, 64, a.seq_len, seed=0) if creator else None
    try:
        with ddl_amd.start(n_producers=2) as (env, conn):
            if env.world_size > 1:
                torch.distributed.barrier(group=env.control_group)
            if src is None:  # other local ranks attach to the creator's segments
                from ddl_amd.models import SharedArraySource

                offs = SharedArraySource(name + "_off", a.n_seqs + 1, (1,), "int64")
                n_tok = int(offs.tensor()[-1])
                src = SharedTokenSource(SharedArraySource(name + "_tok", n_tok, (1,), "int32"), offs, a.seq_len)
            producer = TokenBatchProducer(src, a.global_batch, a.seq_len, a.mode,
                                          pack_order="ffd" if a.mode == "pack" else "in_order",
                                          batches_per_window=a.batches_per_window)
            dl = ddl_amd.DistributedDataLoader(producer, a.global_batch // env.world_size, conn, a.epochs, env=env,
                                               order=ddl_amd.OrderSpec(mode="indexed"),
                                               output=ddl_amd.OutputSpec(collate="tokens"), auto_mark=True)
            for epoch in range(a.epochs):
                real = rows = 0
                for b in dl:
                    real += int(b["attention_mask"].sum())
                    rows += b["input_ids"].shape[0]
                if env.rank == 0:
                    # cu_seqlens has one entry per SEGMENT: over-long sequences are split into seq_len chunks
                    # and empty sequences have none, so this is not the sequence count
                    extra = (f", {b['cu_seqlens'].numel() - 1} segments (max {b['max_seqlen']} tokens) in the "
                             "last batch" if a.mode == "pack" else "")
                    print(f"epoch {epoch}: {rows} rows x {a.seq_len} on rank 0, {real} real tokens "
                          f"({100.0 * real / max(rows * a.seq_len, 1):.1f}% dense){extra}; keys {sorted(b)}",
                          flush=True)
    finally:
        if src is not None:
            src.close()


if __name__ == "__main__":
    main()
