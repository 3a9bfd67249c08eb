#!/usr/bin/env python3
"""Diagnostic: bench.py's world-size-invariant ``indexed`` phase alone, before and after a window-phase loader
has run in the same process (round-3 question: 177-180k inside bench.py vs 188k in bench_zerocopy.py)."""

import json
import math
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(argv=None) -> int:
    import ddl_amd
    from ddl_amd import Marker, ops
    from ddl_amd.models.producers import ImageWindowProducer

    extra = list(sys.argv[1:] if argv is None else argv)  # e.g. --index-no-prefault
    args = bench.parse(["--steps", "200", "--warmup", "20", "--idle-steps", "0", *extra])
    res = {}
    with ddl_amd.start(n_producers=args.producers) as (env, conn):
        dev = torch.device(env.device)

        def sync():
            torch.cuda.synchronize(dev)

        res["indexed_first"] = bench.indexed_phase(args, env, dev, sync, sync)["value"]
        res["indexed_second"] = bench.indexed_phase(args, env, dev, sync, sync)["value"]
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(256, (3, 224, 224), "bfloat16"), 256, conn,
                                           math.ceil(300 / 1) + 1, env=env, device=dev,
                                           output=ddl_amd.OutputSpec(dtype=torch.bfloat16),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=4),
                                           order=ddl_amd.OrderSpec(shuffle="device"))
        acc = ops.ChecksumAccumulator(dev)
        for e in range(300):
            (x,) = dl[0]
            acc.add(x)
            dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
        sync()
        res["indexed_with_window_loader_open"] = bench.indexed_phase(args, env, dev, sync, sync)["value"]
        dl.close()
        res["indexed_after_window_loader"] = bench.indexed_phase(args, env, dev, sync, sync)["value"]
    # bench.py's own window phase (its main, in this process), then the indexed phase again
    bench.main(["--order", "window", "--idle-steps", "0"])
    with ddl_amd.start(n_producers=args.producers) as (env, conn):
        dev = torch.device(env.device)
        res["indexed_after_bench_main"] = bench.indexed_phase(args, env, dev, sync, sync)["value"]
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
