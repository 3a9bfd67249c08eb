#!/usr/bin/env python3
"""Pure-Python share of the consumer's per-batch host cost.

Runs the native-dispatch path (``dl[i]`` + ``mark``) of the reference CI shape with the BatchEngine
replaced by a stub that returns at once (no HIP calls, no kernels). Subtracting this from
``tools/loader_host_cost.py``'s thread CPU time leaves the engine + HIP share. Runs on the CPU
(thread producers); on the GPU box it measures that host's Python speed. Prints one JSON line and
the top of a cProfile.
"""

import collections
import cProfile
import json
import os
import pstats
import sys
import time

os.environ["DDL_DEVICE"] = "cpu"
os.environ["DDL_PRODUCER_MODE"] = "thread"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


class StubEngine:
    """The BatchEngine surface ``DistributedDataLoader`` uses, without HIP."""

    def __init__(self):
        self.n = 0
        self.slots_left = 10 ** 9
        self.inline = True

    def get(self, w, local, bpw, nxt, handle, timeout_ms):
        self.n += 1
        return self.n - 1, -1, (0, 0, 0, 0)

    def release(self, w):
        return 0

    def acquire(self, w, timeout_ms):
        return 0, -1

    def provide(self, ptrs):
        pass


class _Block:
    def record_stream(self, stream):
        pass


class _Stream:
    cuda_stream = 0


def main() -> int:
    import torch

    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.models import PointwiseProducer
    from ddl_amd.utils import streams

    n = 200_000
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(PointwiseProducer(n_timesteps=10, host_shuffle=False), 4096, conn, 10 ** 6,
                                           env=env, order=ddl_amd.OrderSpec(seed=1))
        # the CUDA-only pieces of the fast path, stubbed (after the loader is built: producers are threads)
        torch._C._cuda_getCurrentStream = lambda i: 1
        streams.current = lambda i: _Stream()
        out, block = (torch.empty(1),), _Block()
        dl._engine = StubEngine()
        dl._eng_slots = collections.deque((i, out, block) for i in range(n + 10))
        dl._eng_budget, dl._eng_streams, dl._eng_rec = 0, {}, (None, None)
        dl._eng_window, dl._eng_tokens, dl._eng_whole, dl._eng_block = None, None, False, 64
        dl._engine_provide = lambda: None

        def batches():
            while True:
                for i in range(len(dl)):
                    yield dl[i]
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)

        it = batches()
        for _ in range(1000):
            next(it)
        timed = n - 30_000
        c0 = time.thread_time()
        for _ in range(timed):
            next(it)
        c1 = time.thread_time()
        print(json.dumps({"python_us_per_batch": round(1e6 * (c1 - c0) / timed, 3)}), flush=True)
        prof = cProfile.Profile()
        prof.enable()
        for _ in range(20_000):
            next(it)
        prof.disable()
        pstats.Stats(prof).sort_stats("tottime").print_stats(15)
        sys.stdout.flush()
        dl._engine = None
        os._exit(0)  # thread producers of a 10**6-epoch loader: skip the orderly drain
    return 0


if __name__ == "__main__":
    sys.exit(main())
