#!/usr/bin/env python3
"""Per-kernel throughput of the gfx950 loader kernels at production shapes.

Each kernel is timed with HIP events over many launches and reported as
effective HBM GB/s (bytes read + written) against two denominators: the
8 TB/s HBM3E spec (``pct_of_spec``) and a roofline MEASURED first on the same
box: the best of a 1 GiB device-to-device ``copy_`` and a plain streaming-copy
kernel (``pct_of_d2d``: read + write bytes over its time). A kernel timed in a
loop over one batch-sized buffer (77 MB in, 77 MB out) is partly served by the
256 MB Infinity Cache and can exceed that HBM roofline; the same streaming copy
at that working set is printed as a reference. No child processes, no producers: safe to run under
``rocprofv3 --pmc``.
"""

import json
import sys

import numpy as np
import torch

from ddl_amd import ops
from ddl_amd.permutation import FeistelPermutation


def bench(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


HBM_SPEC_BPS = 8.0e12
D2D_BPS = None  # measured in main()


def report(name, t, bytes_moved, **kw):
    bps = bytes_moved / t
    print(json.dumps({"kernel": name, "us": round(t * 1e6, 2), "GBps": round(bps / 1e9, 1),
                      "pct_of_spec": round(100 * bps / HBM_SPEC_BPS, 1),
                      "pct_of_d2d": round(100 * bps / D2D_BPS, 1) if D2D_BPS else None, **kw}), flush=True)


def measure_d2d() -> float:
    """Measured HBM roofline: the best (bytes read + written) / s of two 1 GiB device-to-device copies,
    the runtime's ``copy_`` (hipMemcpy D2D) and a plain 16 B-per-lane streaming copy kernel
    (``stream_copy``, grid sized 2..16 blocks per CU)."""
    global D2D_BPS
    from ddl_amd import _native

    a = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    best = {}
    t = bench(lambda: b.copy_(a), reps=20)
    best["copy_ (hipMemcpy D2D)"] = t
    hip = _native.hip()
    st = torch.cuda.current_stream().cuda_stream
    for bpc in (2, 4, 8, 16):
        t = bench(lambda: hip.stream_copy(a.data_ptr(), b.data_ptr(), a.numel(), 256 * bpc, st), reps=20)
        best[f"stream_copy {bpc}x256 blocks"] = t
    # one pass: every thread moves 4 x 16 B once (no grid-stride loop); the fastest copy shape measured at
    # 4 GiB by benchmarks/hbm_ceilings.hip (5.69 TB/s), which also gives the read-only / write-only ceilings
    one_shot = a.numel() // 16 // (256 * 4)
    t = bench(lambda: hip.stream_copy(a.data_ptr(), b.data_ptr(), a.numel(), one_shot, st), reps=20)
    best["stream_copy one pass"] = t
    for name, t in best.items():
        bps = 2 * a.numel() / t
        print(json.dumps({"kernel": f"roofline: {name} 1GiB", "us": round(t * 1e6, 2), "GBps": round(bps / 1e9, 1),
                          "pct_of_spec": round(100 * bps / HBM_SPEC_BPS, 1)}), flush=True)
    D2D_BPS = 2 * a.numel() / min(best.values())
    # the same copy at the gathers' working set (77 MB in + 77 MB out): it fits the 256 MB Infinity Cache
    # (MALL) when repeated, which is why kernels on batch-sized buffers can exceed the 1 GiB HBM roofline
    ws = 256 * 3 * 224 * 224 * 2
    for bpc in (2, 4):
        t = bench(lambda: hip.stream_copy(a.data_ptr(), b.data_ptr(), ws, 256 * bpc, st), reps=50)
        print(json.dumps({"kernel": f"reference: stream_copy {bpc}x256 blocks 77MB (batch working set)",
                          "us": round(t * 1e6, 2), "GBps": round(2 * ws / t / 1e9, 1),
                          "pct_of_spec": round(100 * 2 * ws / t / HBM_SPEC_BPS, 1),
                          "pct_of_d2d": round(100 * 2 * ws / t / D2D_BPS, 1)}), flush=True)
    return D2D_BPS


def main():
    dev = torch.device("cuda", 0)
    measure_d2d()
    B, C, H, W = 256, 3, 224, 224
    n = 2048
    win_bf16 = torch.randn(n, C, H, W, device=dev).to(torch.bfloat16)
    win_u8 = torch.randint(0, 256, (n, C, H, W), dtype=torch.uint8, device=dev)
    win_hwc = torch.randint(0, 256, (n, H, W, C), dtype=torch.uint8, device=dev)
    p = FeistelPermutation(n, 1, 2)
    out_bf16 = torch.empty(B, C, H, W, dtype=torch.bfloat16, device=dev)
    img = C * H * W
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    sc = [1 / (255 * s_) for s_ in std]
    bi = [-m / s_ for m, s_ in zip(mean, std)]

    t = bench(lambda: ops.gather_rows(win_bf16, perm=p, base=0, n_rows=B, out=out_bf16))
    report("permute_gather bf16->bf16", t, 2 * B * img * 2, rows=B, row_bytes=img * 2)
    t = bench(lambda: ops.gather_rows(win_u8, perm=p, base=0, n_rows=B, out=out_bf16, scale=sc, bias=bi,
                                      plane=H * W))
    report("permute_gather u8->bf16 normalise", t, B * img * 3, rows=B)
    t = bench(lambda: ops.collate_hwc_to_chw(win_hwc, perm=p, base=0, n_rows=B, out=out_bf16, mean=mean, std=std))
    report("collate HWC u8 -> CHW bf16 normalise", t, B * img * 3, rows=B)
    f32 = torch.randn(B, img, device=dev)
    t = bench(lambda: ops.cast(f32, torch.bfloat16))
    report("cast f32->bf16", t, B * img * 6)
    idx = torch.from_numpy(p(np.arange(B))).to(dev)
    t = bench(lambda: ops.scatter_rows(win_bf16.view(n, -1), out_bf16.view(B, -1), idx))
    report("scatter_rows bf16", t, 2 * B * img * 2)
    t = bench(lambda: ops.checksum(out_bf16))
    report("checksum (reduce)", t, B * img * 2)
    cacc = ops.ChecksumAccumulator(dev)
    t = bench(lambda: cacc.add(out_bf16))
    report("checksum accumulate (streaming consumer)", t, B * img * 2)
    t = bench(lambda: ops.feistel_indices(FeistelPermutation(1 << 24, 3, 3), 0, 1 << 24, device=dev), reps=10)
    report("feistel_indices 16M", t, (1 << 24) * 8)
    # augmentation: RandomResizedCrop 256x320 u8 -> 224x224 bf16 (+ flip + normalise), CHW and HWC sources
    for layout in ("chw", "hwc"):
        shp = (1024, 3, 256, 320) if layout == "chw" else (1024, 256, 320, 3)
        raw = torch.randint(0, 255, shp, dtype=torch.uint8, device=dev)
        p1k = FeistelPermutation(1024, 1, 3)
        t = bench(lambda: ops.random_resized_crop(raw, perm=p1k, base=0, n_rows=B, size=(224, 224), seed=1,
                                                  layout=layout, mean=[0.5] * 3, std=[0.25] * 3))
        report(f"random_resized_crop {layout} u8 256x320 -> bf16 224x224", t, B * img * 2)
    # pointwise (reference CI shape): 100,520 x 9 f32 window, 4096-row batch split (3,5,1)
    pw = torch.randn(100_520, 9, device=dev)
    pp = FeistelPermutation(100_520, 5, 5)
    t = bench(lambda: ops.split_columns(pw, (3, 5, 1), perm=pp, base=0, n_rows=4096))
    report("split_columns 4096x(3,5,1) f32", t, 2 * 4096 * 36)
    # whole-window dispatch: the window's 24 batches in one launch (same kernel, 24x the rows)
    t = bench(lambda: ops.split_columns(pw, (3, 5, 1), perm=pp, base=0, n_rows=24 * 4096))
    report("split_columns 24x4096x(3,5,1) f32 (one launch per window)", t, 2 * 24 * 4096 * 36)
    # resident exchange bucketing (W=8, global batch 2048): send list + receive map, one workgroup each
    from ddl_amd import _native

    hip = _native.hip()
    pr = FeistelPermutation(1 << 20, 7, 1)
    S, W, GB, LB, rank = (1 << 20) // 8, 8, 2048, 256, 1
    send_idx = torch.empty(GB, dtype=torch.int64, device=dev)
    inv_idx = torch.empty(LB, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    send_c, recv_c = _native.runtime().owner_counts(pr.keys, pr.half_bits, pr.n, 0, GB, LB, S, W, rank)
    t = bench(lambda: hip.bucket_send(pr.keys, pr.n, pr.half_bits, 0, GB, S, S * rank, rank, W,
                                      send_idx.data_ptr(), st))
    report("bucket_send W=8 GB=2048", t, GB * 8, sent=sum(send_c))
    offs = [0]
    for c in recv_c[:-1]:
        offs.append(offs[-1] + c)
    t = bench(lambda: hip.bucket_recv(pr.keys, pr.n, pr.half_bits, rank * LB, LB, S, W, offs,
                                      inv_idx.data_ptr(), st))
    report("bucket_recv W=8 slice 256", t, LB * 8)
    grp = [pw[:, :3].contiguous(), pw[:, 3:8].contiguous(), pw[:, 8:].contiguous()]
    t = bench(lambda: ops.pack_columns(grp))
    report("pack_columns window 100520x(3,5,1) f32", t, 2 * 100_520 * 36)
    t = bench(lambda: ops.pack_columns(grp, perm=pp, base=0, n_rows=4096, out_dtype=torch.bfloat16))
    report("pack_columns 4096 gather+bf16", t, 4096 * 36 + 4096 * 18)
    # tokens: 64 sequences, mean 2k, seq_len 4096 pack + pad
    rng = np.random.default_rng(0)
    lens = rng.integers(256, 4097, size=64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    toks = torch.from_numpy(rng.integers(0, 50000, size=int(offs[-1])).astype(np.int32)).to(dev)
    offs_d = torch.from_numpy(offs).to(dev)
    t = bench(lambda: ops.pad_tokens(toks, offs_d, 4096))
    report("pad_tokens 64x4096", t, toks.numel() * 4 + 64 * 4096 * (4 + 1 + 8))
    t = bench(lambda: ops.pack_tokens(toks, offs, 4096), reps=20)
    report("pack_tokens 64 seqs (incl. host plan)", t, toks.numel() * (4 + 4 + 1 + 8 + 4))
    # the plan on the device: plan kernel + pack kernel reading the row count from device memory (no host
    # round trip; static shapes), output rows = pack_capacity
    t = bench(lambda: ops.pack_tokens_device(toks, offs_d, 4096), reps=20)
    report("pack_tokens 64 seqs (device plan, 2 launches)", t, toks.numel() * (4 + 4 + 1 + 8 + 4))
    lens2 = rng.integers(1, 4097, size=2048)
    offs2 = torch.from_numpy(np.concatenate([[0], np.cumsum(lens2)]).astype(np.int64)).to(dev)
    toks2 = torch.from_numpy(rng.integers(0, 50000, size=int(lens2.sum())).astype(np.int32)).to(dev)
    t = bench(lambda: ops.pack_tokens_device(toks2, offs2, 4096), reps=20)
    report("pack_tokens 2048 seqs (device plan, 2 launches)", t, toks2.numel() * (4 + 4 + 1 + 8 + 4))
    t = bench(lambda: ops.pack_tokens(toks2, offs2.cpu().numpy(), 4096), reps=10)
    report("pack_tokens 2048 seqs (incl. host plan)", t, toks2.numel() * (4 + 4 + 1 + 8 + 4))
    # the same two launches captured in a HIP graph: device time only (no Python / allocator on the host)
    for name, (tk, of) in (("64", (toks, offs_d)), ("2048", (toks2, offs2))):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ops.pack_tokens_device(tk, of, 4096)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ops.pack_tokens_device(tk, of, 4096)
        t = bench(g.replay, reps=20)
        report(f"pack_tokens {name} seqs (device plan, graph replay)", t, tk.numel() * (4 + 4 + 1 + 8 + 4))
    x = torch.randn(1_000_000, 9, device=dev)
    t = bench(lambda: ops.column_stats(x), reps=20)
    report("column_stats 1Mx9", t, x.numel() * 4)
    del win_bf16, win_u8, win_hwc, raw, pw, x
    out_of_cache(dev)


def rotating(fns, reps=48):
    """Time a list of calls issued round-robin (each touches its own buffers), per call."""
    i = [0]

    def one():
        fns[i[0] % len(fns)]()
        i[0] += 1

    return bench(one, reps=reps)


def out_of_cache(dev) -> None:
    """The gather / cast / scatter kernels on working sets far beyond the 256 MB MALL: 1024-row batches
    from an 8192-image window (2.5 GB bf16 / 1.2 GB uint8), 4 output buffers used round-robin, so every
    call reads and writes memory the previous calls did not touch (>= 1.2 GB in flight per rotation).
    These are the numbers to hold against the 1 GiB D2D roofline (``pct_of_d2d``)."""
    B, C, H, W, n = 1024, 3, 224, 224, 8192
    img = C * H * W
    p = FeistelPermutation(n, 1, 2)
    win = torch.empty(n, C, H, W, dtype=torch.bfloat16, device=dev).normal_()
    outs = [torch.empty(B, C, H, W, dtype=torch.bfloat16, device=dev) for _ in range(4)]
    fns = [lambda o=o, k=k: ops.gather_rows(win, perm=p, base=k * B, n_rows=B, out=o) for k, o in enumerate(outs)]
    report("OOC permute_gather bf16->bf16 1024 rows (rotating)", rotating(fns), 2 * B * img * 2, rows=B)
    idxs = [torch.from_numpy(p(np.arange(k * B, (k + 1) * B))).to(dev) for k in range(4)]
    fns = [lambda o=o, ix=ix: ops.scatter_rows(win.view(n, -1), o.view(B, -1), ix) for o, ix in zip(outs, idxs)]
    report("OOC scatter_rows bf16 1024 rows (rotating)", rotating(fns), 2 * B * img * 2, rows=B)
    del win
    win8 = torch.randint(0, 256, (n, C, H, W), dtype=torch.uint8, device=dev)
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    sc = [1 / (255 * s_) for s_ in std]
    bi = [-m / s_ for m, s_ in zip(mean, std)]
    fns = [lambda o=o, k=k: ops.gather_rows(win8, perm=p, base=k * B, n_rows=B, out=o, scale=sc, bias=bi,
                                            plane=H * W) for k, o in enumerate(outs)]
    report("OOC permute_gather u8->bf16 normalise 1024 rows (rotating)", rotating(fns), B * img * 3, rows=B)
    del win8
    f32s = [torch.empty(B, img, device=dev).normal_() for _ in range(2)]
    fns = [lambda f=f, o=o: ops.gather_rows(f, out=o.view(B, img)) for f, o in zip(f32s * 2, outs)]
    report("OOC cast f32->bf16 1024 rows (rotating)", rotating(fns), B * img * 6, rows=B)


if __name__ == "__main__":
    sys.exit(main())
