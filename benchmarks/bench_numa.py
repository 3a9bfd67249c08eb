#!/usr/bin/env python3
"""GPU reads of pinned host memory from the GPU's own NUMA node vs. a remote one.

The reference keeps each GPU group's data in node-local shared memory (reference
ddl/ddl_env.py:58-73, ddl/connection.py:88-139). On a 2-socket 8-GPU MI355X node, memory on the
other socket adds the inter-socket link to every PCIe read. For each NUMA node of this host that
has memory, a shm segment is bound to that node (mbind, strict), filled, page placement verified
(move_pages), registered with the GPU, and read two ways:

* ``sdma``: ``hipMemcpyAsync`` H2D of whole windows (the stager's path), two copy streams;
* ``zerocopy``: the ``ZeroCopyLoader`` gather kernel (the world-size-invariant ``indexed`` phase of
  bench.py): one kernel per batch gathers 256 Feistel-permuted 3x224x224 bf16 samples over PCIe.

One JSON line per node; ``local`` marks the GPU's node.
"""

import argparse
import json
import os
import sys
import time


def _nodes_with_memory() -> list[int]:
    base = "/sys/devices/system/node"
    out = []
    for d in sorted(os.listdir(base)):
        if d.startswith("node") and d[4:].isdigit():
            try:
                with open(os.path.join(base, d, "meminfo")) as f:
                    total = next((int(ln.split()[3]) for ln in f if "MemTotal" in ln), 0)
            except (OSError, StopIteration, ValueError):
                total = 0
            if total > 0:
                out.append(int(d[4:]))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--samples", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--copies", type=int, default=60, help="H2D window copies per node (sdma)")
    ap.add_argument("--window", type=int, default=256)
    a = ap.parse_args(argv)

    import torch

    from ddl_amd import _native, ops
    from ddl_amd.models.datasets import SharedArraySource
    from ddl_amd.utils.numa import gpu_numa_node
    from ddl_amd.zerocopy import ZeroCopyLoader

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gnode = gpu_numa_node(0)
    hip = _native.hip()
    shape = (3, 224, 224)
    nodes = _nodes_with_memory()
    print(json.dumps({"gpu_numa_node": gnode, "nodes_with_memory": nodes, "cpus": len(os.sched_getaffinity(0))}),
          flush=True)
    for node in nodes:
        name = f"ddl_amd_numa_{os.getpid()}_{node}"
        src = SharedArraySource(name, a.samples, shape, torch.bfloat16, create=True)
        rec = {"node": node, "local": node == gnode}
        try:
            rc = src.bind_to_node(node, strict=True)
            rec["mbind_rc"] = rc
            t = src.tensor()
            t.view(torch.uint8).fill_(0x3C)
            t.view(a.samples, -1)[:, 0] = torch.arange(a.samples, dtype=torch.float32).to(torch.bfloat16)
            pages = src.page_nodes(256)
            rec["pages_on_node_pct"] = round(100.0 * sum(1 for p in pages if p == node) / len(pages), 1)

            # sdma: window-sized H2D copies out of the registered segment, alternating two streams
            win_bytes = a.window * src.row_bytes
            base = src.address & ~4095
            size = -(-(src.address + a.samples * src.row_bytes - base) // 4096) * 4096
            hip.host_register(base, size, True)
            try:
                dsts = [torch.empty(win_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
                ss = [torch.cuda.Stream(dev) for _ in range(2)]
                n_win = a.samples // a.window

                def copies(k):
                    for i in range(k):
                        off = (i % n_win) * win_bytes
                        hip.memcpy_h2d(dsts[i % 2].data_ptr(), src.address + off, win_bytes, ss[i % 2].cuda_stream)

                copies(8)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                copies(a.copies)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                rec["sdma_gbps"] = round(a.copies * win_bytes / el / 1e9, 2)
                rec["sdma_samples_per_s"] = round(a.copies * a.window / el, 1)
            finally:
                torch.cuda.synchronize()
                hip.host_unregister(base)

            # zero-copy gather kernel (registers the segment itself)
            dl = ZeroCopyLoader(src, a.batch, seed=1, out_dtype=torch.bfloat16, device=dev)
            acc = ops.ChecksumAccumulator(dev)
            it = iter(dl)
            for _ in range(10):
                acc.add(next(it))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                try:
                    x = next(it)
                except StopIteration:
                    it = iter(dl)
                    x = next(it)
                acc.add(x)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            dl.close()
            rec["zerocopy_samples_per_s"] = round(a.batch * a.steps / el, 1)
            rec["zerocopy_gbps"] = round(a.batch * a.steps * src.row_bytes / el / 1e9, 2)
        finally:
            src.close()
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
