#!/usr/bin/env python3
"""Calibrate the host->HBM paths the loader can use on this box.

* SDMA copies (hipMemcpyAsync H2D) out of a hipHostRegister'ed shm arena: GB/s
  vs copy size and number of concurrent streams;
* zero-copy kernel gather (gfx950 gather_rows reading device-mapped host
  memory over PCIe);
* HBM->HBM Feistel-permutation gather of 301 KB image rows (+ bf16 cast).
Prints one JSON line per measurement.
"""

import json
import time

import torch

from ddl_amd import _native, ops
from ddl_amd.permutation import FeistelPermutation


def timed(fn, reps=10, streams=()):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    rt, h = _native.runtime(), _native.hip()
    total = 2 << 30
    a = rt.Arena.create("/ddl_amd.probe", [total], 1)
    a.unlink()
    h.host_register(a.base_address, a.total_bytes, True)
    host = torch.frombuffer(a.slot_view(0, 0), dtype=torch.uint8)
    host[:] = 7
    dev = torch.device("cuda", 0)
    dst = torch.empty(total, dtype=torch.uint8, device=dev)
    src_addr = a.slot_address(0, 0)
    for nstreams in (1, 2, 4):
        ss = [torch.cuda.Stream() for _ in range(nstreams)]
        for size in (16 << 20, 64 << 20, 256 << 20, 1 << 30):
            per = size // nstreams

            def go():
                for i, s in enumerate(ss):
                    h.memcpy_h2d(dst.data_ptr() + i * per, src_addr + i * per, per, s.cuda_stream)

            t = timed(go, reps=5)
            print(json.dumps({"probe": "sdma_h2d", "streams": nstreams, "bytes": size, "GBps": round(size / t / 1e9, 2)}))
    # pageable (plain torch cpu tensor) for comparison
    pg = torch.empty(256 << 20, dtype=torch.uint8)
    t = timed(lambda: dst[: 256 << 20].copy_(pg, non_blocking=True), reps=5)
    print(json.dumps({"probe": "torch_copy_pageable", "bytes": 256 << 20, "GBps": round((256 << 20) / t / 1e9, 2)}))
    # zero-copy kernel gather from mapped host memory
    row = 3 * 224 * 224 * 2
    n = total // row
    rows_h = ops.HostRows(host[: n * row].view(n, row), h.host_device_pointer(src_addr))
    out = torch.empty((256, row), dtype=torch.uint8, device=dev)
    p = FeistelPermutation(n, 1, 1)
    t = timed(lambda: ops.gather_rows(rows_h, perm=p, base=0, n_rows=256, out=out), reps=10)
    print(json.dumps({"probe": "zero_copy_gather", "rows": 256, "row_bytes": row, "GBps": round(256 * row / t / 1e9, 2)}))
    # HBM->HBM permutation gather (bf16 rows)
    hb = dst[: n * row].view(n, row // 2 * 2).view(torch.bfloat16).view(n, -1)
    outb = torch.empty((256, hb.shape[1]), dtype=torch.bfloat16, device=dev)
    t = timed(lambda: ops.gather_rows(hb, perm=p, base=0, n_rows=256, out=outb), reps=50)
    print(json.dumps({"probe": "hbm_perm_gather_bf16", "rows": 256, "GBps_rw": round(2 * 256 * row / t / 1e9, 1), "us": round(t * 1e6, 1)}))
    u8 = dst[: n * (row // 2)].view(n, row // 2)
    t = timed(lambda: ops.gather_rows(u8, perm=p, base=0, n_rows=256, out_dtype=torch.bfloat16,
                                      scale=[1 / 58.0] * 3, bias=[-2.0] * 3, plane=224 * 224), reps=50)
    print(json.dumps({"probe": "hbm_perm_gather_u8_to_bf16_norm", "rows": 256, "us": round(t * 1e6, 1),
                      "GBps_rw": round(256 * (row // 2) * 3 / t / 1e9, 1)}))
    t = timed(lambda: ops.checksum(outb), reps=50)
    print(json.dumps({"probe": "checksum_77MB", "us": round(t * 1e6, 1), "GBps": round(outb.numel() * 2 / t / 1e9, 1)}))
    h.host_unregister(a.base_address)


if __name__ == "__main__":
    main()
