"""Host-side cost (µs per call) of the pieces on the loader's per-batch path (GPU box)."""
import json
import time

import torch

from ddl_amd import ops
from ddl_amd.permutation import FeistelPermutation


def t(fn, n=20000):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    return round(dt, 2)


dev = torch.device("cuda", 0)
bs = torch.cuda.Stream(dev)
cur = torch.cuda.current_stream(dev)
ev = torch.cuda.Event()
ev.record(bs)
x = torch.empty(4096, 9, device=dev)
win = torch.randn(100_520, 9, device=dev)
perm = FeistelPermutation(100_520, 1, 2)
acc = ops.ChecksumAccumulator(dev)
out = {}
out["Event()"] = t(lambda: torch.cuda.Event())
out["ev.record(bs)"] = t(lambda: ev.record(bs))
out["Event().record(bs) (new hipEvent each call)"] = t(lambda: torch.cuda.Event().record(bs))
# re-recording the SAME event with nothing enqueued in between is a fast path (~1.4 us); a ring of
# pre-created events costs as much as a fresh one (~6 us): the price is the marker, not the creation
ring = [torch.cuda.Event() for _ in range(8)]
_k = [0]


def ring_record():
    _k[0] = (_k[0] + 1) % 8
    ring[_k[0]].record(bs)


out["ring of 8 events .record(bs)"] = t(ring_record)
out["cur.wait_event"] = t(lambda: cur.wait_event(ev))
out["bs.wait_event"] = t(lambda: bs.wait_event(ev))


def ctx():
    with torch.cuda.stream(bs):
        pass


out["with torch.cuda.stream(bs)"] = t(ctx)
out["current_stream(dev)"] = t(lambda: torch.cuda.current_stream(dev))
out["x.record_stream(cur)"] = t(lambda: x.record_stream(cur))
out["torch.empty 4096x3"] = t(lambda: torch.empty((4096, 3), device=dev))
out["split_columns 3 groups"] = t(lambda: ops.split_columns(win, (3, 5, 1), perm=perm, base=0, n_rows=4096), 5000)
out["gather_rows perm"] = t(lambda: ops.gather_rows(win, perm=perm, base=0, n_rows=4096), 5000)
out["checksum acc.add"] = t(lambda: acc.add(x), 5000)
out["perm.device_args()"] = t(lambda: perm.device_args())
print(json.dumps(out))
