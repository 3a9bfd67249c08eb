#!/usr/bin/env python3
"""Host cost of the HBM-resident loader's W > 1 step, rehearsed at W = 8 over gloo on the CPU.

Eight rank processes (``tests/mp_harness.run_ranks``, gloo, 127.0.0.1) each hold a shard of a
node-shared synthetic source and iterate ``ResidentGlobalLoader``; rank 0 runs the steps under
cProfile. Per step the loader computes the W split counts (native Feistel, ``owner_counts``), the
send list and the receive map (``bucket.hip`` on a GPU; here their native host twin ``owner_maps``),
gathers, runs the all-to-all and gathers the batch. The report lists the per-step host time and the
profile's top entries by cumulative time, and checks that no numpy routine (``np.argsort``,
``np.bincount``, ``np.nonzero``, ...) is on the step's path any more.
"""

from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def _rank(rank, world, name, n, gb, steps, out_dir):
    import cProfile
    import io
    import pstats
    import time

    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    src = SharedArraySource(name, n, (64,), "float32")
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ResidentGlobalLoader(src, gb, env, seed=3, depth=2, device="cpu")
        it = iter(dl)
        for _ in range(5):
            next(it)
        prof = cProfile.Profile() if rank == 0 else None
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        for _ in range(steps):
            try:
                next(it)
            except StopIteration:
                it = iter(dl)
                next(it)
        if prof:
            prof.disable()
        dt = (time.perf_counter() - t0) / steps
        res = {"rank": rank, "host_ms_per_step": round(1e3 * dt, 3)}
        if prof:
            s = io.StringIO()
            st = pstats.Stats(prof, stream=s).sort_stats("cumulative")
            st.print_stats(30)
            text = s.getvalue()
            with open(os.path.join(out_dir, "rank0_profile.txt"), "w") as f:
                f.write(text)
            numpy_calls = sorted({f"{fn[2]}" for fn in st.stats if "numpy" in fn[0] and fn[2] in
                                  ("argsort", "bincount", "nonzero", "unique", "searchsorted", "cumsum", "concatenate")})
            res["numpy_on_step_path"] = numpy_calls
        return res


def main() -> int:
    import numpy as np
    import torch

    from ddl_amd.models import SharedArraySource
    from tests.mp_harness import run_ranks

    out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/resident_w8"
    os.makedirs(out_dir, exist_ok=True)
    n, gb, steps, world = 64_000, 2048, 60, 8
    src = SharedArraySource.create(f"ddl_amd_rsp_{np.random.randint(1 << 30)}",
                                   torch.arange(n * 64, dtype=torch.float32).view(n, 64))
    try:
        res = run_ranks(_rank, world, src.name, n, gb, steps, out_dir, timeout=600)
    finally:
        src.close()
    line = {"world": world, "global_batch": gb, "steps": steps, "backend": "gloo (CPU rehearsal)",
            "host_ms_per_step_max": max(r["host_ms_per_step"] for r in res),
            "numpy_on_step_path": res[0].get("numpy_on_step_path"), "per_rank": res}
    print(json.dumps(line))
    with open(os.path.join(out_dir, "resident_w8.json"), "w") as f:
        f.write(json.dumps(line) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
