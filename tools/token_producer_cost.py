#!/usr/bin/env python3
"""Host cost of one token producer round (config 4 shape: 64 sequences of mean ~2.2k tokens per batch,
seq_len 4096, FFD packing, k batches per window), in-process, no loader: per-batch microseconds of
``TokenBatchProducer.execute_function`` for 1, 2 and 4 gather threads, and the top of a cProfile.
"""

import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main() -> int:
    import torch

    from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer

    k = int(os.environ.get("K", "8"))
    src = SharedTokenSource.synthetic(f"ddl_amd_tpc_{os.getpid()}", 8192, 256, 4096, seed=1)
    try:
        for threads in (1, 2, 4):
            p = TokenBatchProducer(src, 64, 4096, "pack", pack_order="ffd", batches_per_window=k,
                                   host_threads=threads)
            p.producer_index, p.n_producers, p.rank_global = 0, 4, 0
            ret = p.on_init(world_size=1, seed=0)
            buf = torch.empty(ret.shape[0] * ret.shape[1], dtype=torch.uint8)
            for r in range(5):
                p.execute_function(round=r, my_tensor=buf)
            n = 100
            t0 = time.perf_counter()
            for r in range(n):
                p.execute_function(round=r, my_tensor=buf)
            dt = (time.perf_counter() - t0) / n
            print(json.dumps({"host_threads": threads, "k": k, "us_per_window": round(dt * 1e6, 1),
                              "us_per_batch": round(dt * 1e6 / k, 1)}), flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for r in range(50):
            p.execute_function(round=r, my_tensor=buf)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(10)
        print(s.getvalue())
    finally:
        src.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
