"""Debug: IndexedProducer over a uint8 .npy, native inline / lookahead vs Python dispatch, per-batch diff."""
import sys
import tempfile

import numpy as np
import torch

import ddl_amd
from ddl_amd.models import FileRowsSource, IndexedProducer
from ddl_amd.permutation import EpochOrder


def run(src, gb, native):
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, gb), gb, conn, 1, env=env, auto_mark=True,
                                           staging=ddl_amd.StagingSpec(native_dispatch=native),
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=5))
        out = [b[0].cpu().numpy().copy() for b in dl]
    return out


def main():
    n, gb = 3000, 128
    arr = np.random.default_rng(0).integers(0, 255, size=(n, 3, 8, 8), dtype=np.uint8)
    with tempfile.TemporaryDirectory() as d:
        path = d + "/imgs.npy"
        np.save(path, arr)
        for direct in (False, True):
            src = FileRowsSource.from_npy(path, direct=direct)
            order = EpochOrder(n, gb, 5)
            ref = arr[order.perm(0).full()[: order.batches_per_epoch * gb]].reshape(-1, gb, 3, 8, 8)
            for native in (False, "inline", "lookahead"):
                got = run(src, gb, native)
                bad = [i for i, (g, r) in enumerate(zip(got, ref)) if not np.array_equal(g, r)]
                rows = {i: int((got[i] != ref[i]).reshape(gb, -1).any(1).sum()) for i in bad}
                print(f"direct={direct} native={native}: {len(got)} batches, bad {bad} bad-rows {rows}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
