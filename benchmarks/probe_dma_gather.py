#!/usr/bin/env python3
"""SDMA row gather vs the zero-copy gather kernel for a world-size-invariant (random) batch order.

``ZeroCopyLoader`` reads a batch's rows out of pinned host memory with a kernel (PCIe reads by CUs, ~54
GB/s in the bench's indexed phase). The alternative is one SDMA copy per row (``dma_gather_rows``:
hipMemcpyAsync per run of consecutive rows; ``hipMemcpyBatchAsync`` when the HIP runtime has it). This
probe times both for 256 random rows of 3x224x224 bf16 (301 KB) from a 4096-row pinned source: device
GB/s over 20 batches, and host µs per batch spent enqueueing.
"""

import json
import time

import numpy as np
import torch

from ddl_amd import _native, ops


def main() -> int:
    dev = torch.device("cuda", 0)
    hip = _native.hip()
    n, rows, shape = 4096, 256, (3, 224, 224)
    src = torch.empty((n,) + shape, dtype=torch.bfloat16, pin_memory=True)
    src.view(torch.uint8).fill_(0x3C)
    row_bytes = src[0].numel() * 2
    out = torch.empty((rows,) + shape, dtype=torch.bfloat16, device=dev)
    rng = np.random.default_rng(0)
    idx = [rng.permutation(n)[:rows].astype(np.int64) for _ in range(20)]
    s = torch.cuda.Stream(dev)
    res = {"has_memcpy_batch": bool(hip.has_memcpy_batch()), "row_bytes": row_bytes, "rows": rows}
    for mode in ("loop", "batched"):
        if mode == "batched" and not res["has_memcpy_batch"]:
            continue
        host_ns = 0
        for rep in range(2):  # the first pass warms the engines
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            host_ns = 0
            for k in range(20):
                host_ns += hip.dma_gather_rows(out.data_ptr(), src.data_ptr(), row_bytes, idx[k].ctypes.data, rows,
                                               n, s.cuda_stream, mode == "batched")
            s.synchronize()
            dt = time.perf_counter() - t0
        res[f"dma_{mode}_GBps"] = round(20 * rows * row_bytes / dt / 1e9, 2)
        res[f"dma_{mode}_host_us_per_batch"] = round(host_ns / 20 / 1e3, 1)
        ref = src[torch.from_numpy(idx[-1])]
        res[f"dma_{mode}_exact"] = bool(torch.equal(out.cpu(), ref))
    dptr = hip.host_device_pointer(src.data_ptr())
    hr = ops.HostRows(src, dptr)
    for cap in (32, 0):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(20):
                ops.gather_rows(hr, index=torch.from_numpy(idx[k]).to(dev), n_rows=rows, max_blocks=cap)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        res[f"zero_copy_kernel_cap{cap}_GBps"] = round(20 * rows * row_bytes / dt / 1e9, 2)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
