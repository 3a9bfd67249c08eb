"""Lean HIP-stream helpers for the per-batch host path.

``torch.cuda.stream(s)`` costs ~7 us per enter/exit and
``torch.cuda.current_stream(dev)`` ~3 us on the MI355X box
(``tools/host_overhead.py``): both rebuild ``Stream`` objects and resolve
devices in Python. The loader switches streams and queries the current
stream once per batch, so these helpers go straight to the C++ stream
registry (same semantics, same-device only).
"""

from __future__ import annotations

import torch

_cache: dict = {}


def current(device_index: int) -> torch.cuda.Stream:
    """``torch.cuda.current_stream(device_index)`` with the Stream object cached per stream id."""
    sid = torch._C._cuda_getCurrentStream(device_index)
    s = _cache.get(sid)
    if s is None:
        s = _cache[sid] = torch.cuda.Stream(stream_id=sid[0], device_index=sid[1], device_type=sid[2])
    return s


class on_stream:  # noqa: N801  (used like torch.cuda.stream)
    """``with on_stream(s):`` makes ``s`` current on its device and restores the previous stream.

    ``s`` must be on the current device (the loader's streams always are).
    """

    __slots__ = ("s", "prev")

    def __init__(self, s: torch.cuda.Stream):
        self.s = s
        self.prev = None

    def __enter__(self):
        s = self.s
        self.prev = torch._C._cuda_getCurrentStream(s.device_index)
        torch._C._cuda_setStream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *exc):
        p = self.prev
        torch._C._cuda_setStream(stream_id=p[0], device_index=p[1], device_type=p[2])
        return False


def batch_stream(device) -> torch.cuda.Stream:
    """The stream the loader builds batches on, at HIGH priority.

    A batch kernel (gather / cast / collate, tens of microseconds) runs next to the training
    step's GEMMs, which occupy every CU. At normal priority the dispatcher only gets to its
    workgroups when the step's kernels drain, so the next step waits for it; a high-priority
    hardware queue has its workgroups dispatched as soon as any CU frees up.
    """
    try:
        _, hi = torch.cuda.Stream.priority_range()  # (least, greatest); greatest is the most negative
    except Exception:  # pragma: no cover - older torch
        hi = -1
    return torch.cuda.Stream(device, priority=hi)
