"""Producer-free zero-copy loader: a gfx950 kernel gathers each batch straight out
of pinned, device-mapped host memory over PCIe.

The window/indexed loaders move data host->HBM with SDMA copies of buffers
that host producers assembled (a host memcpy per sample). For a dataset that
already sits in host memory (node-shared shm, an ``.npy`` memmap in the page
cache, a pinned tensor), there is a shorter MI355X path:

* the whole source is registered once with ``hipHostRegister(..., Mapped)``;
* per step, ONE ``gather_rows`` kernel evaluates the world-size-invariant
  Feistel permutation inline, reads this rank's samples directly over PCIe
  (16 B/lane loads of the mapped host pages) and writes the bf16 batch --
  fused with the dtype cast / per-channel normalisation -- into HBM;
* no producer processes, no host memcpy, no staging buffers, no per-sample
  host work at all;
* the kernel is PCIe-latency-bound, not CU-bound: ~2 us x ~55 GB/s is ~110 KB
  in flight, i.e. a few dozen waves. ``max_blocks`` caps its grid
  (grid-stride over row tiles) so it occupies a handful of CUs and the
  training step keeps the rest; it runs ``depth`` steps ahead on its own
  stream.

Same order and checkpoint format as ``IndexedProducer`` / ``ResidentGlobalLoader``
(``kind="indexed"``), so runs can switch between the three paths on resume.
"""

from __future__ import annotations

from typing import Any

import torch

from . import _native, ops
from .ops import _dtypes
from .permutation import EpochOrder
from .resident import PrefetchedIndexedLoader, _source_address, _source_geometry
from .types import DDLEnv
from .utils import streams

_PAGE = 4096


def _cpu_view(source, n: int, shape, dtype) -> torch.Tensor:
    if isinstance(source, torch.Tensor):
        return source
    if hasattr(source, "tensor"):
        return source.tensor()
    import numpy as np

    a = source._a()
    return torch.from_numpy(np.asarray(a)).view(dtype).view((n,) + tuple(shape))


class ZeroCopyLoader(PrefetchedIndexedLoader):
    def __init__(self, source, global_batch: int, env: DDLEnv | None = None, *, seed: int = 0,
                 drop_last: bool = True, out_dtype: Any = None, normalize: dict | None = None, depth: int = 2,
                 max_blocks: int | None = None, device: str | torch.device | None = None,
                 n_epochs: int | None = None,
                 resume_state: dict | None = None, prep_streams: int = 1, prefault: bool = True,
                 handoff: str = "host"):
        if handoff not in ("host", "device"):
            raise ValueError("handoff must be 'host' or 'device'")
        self.handoff = handoff  # PCIe-paced batches (~1.4 ms each): no barrier packet in the caller's queue
        self.env = env or DDLEnv()
        self.W, self.rank = self.env.world_size, self.env.rank
        self.sample_shape, self.src_dtype = _source_geometry(source)
        addr, n = _source_address(source)
        if not drop_last:  # the device-side order covers whole global batches only
            raise ValueError(f"{type(self).__name__} needs drop_last=True")
        self.order = EpochOrder(n, global_batch, seed, drop_last)
        self.GB, self.LB = int(global_batch), self.order.local_batch(self.W)
        self.out_dtype = _dtypes.to_torch_dtype(out_dtype) if out_dtype is not None else self.src_dtype
        self.normalize = normalize
        if max_blocks is None:
            # measured grid caps (archive/profiles/r1_zerocopy, archive/profiles/r2_misc): a same-width copy is
            # PCIe-bound and peaks at 32 workgroups (bf16: 188k vs 182k samples/s at 64); a widening uint8 -> bf16
            # gather writes twice the bytes it reads and keeps improving up to the full grid
            src_bytes = torch.empty((), dtype=self.src_dtype).element_size()
            out_bytes = torch.empty((), dtype=self.out_dtype).element_size()
            max_blocks = 32 if out_bytes <= src_bytes else 0
        self.max_blocks = int(max_blocks)
        if device is None:
            device = self.env.device or ("cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._init_cursor(seed, depth, n_epochs, resume_state)
        self.cpu = _cpu_view(source, n, self.sample_shape, self.src_dtype)
        self._source = source  # keep the mapping alive
        row_bytes = self.cpu[0].numel() * self.cpu.element_size() if n else 0
        self.nbytes = n * row_bytes
        self._reg_base = None
        self.prep_stream = None
        if self.device.type == "cuda":
            hip = _native.hip()
            if isinstance(source, torch.Tensor):
                # A heap tensor shares its edge pages with unrelated allocations: registering
                # the page-rounded range would pin (and mark as registered) memory that other
                # host buffers live in. Use a pinned copy instead (hipHostMalloc'd, mapped).
                if not self.cpu.is_pinned():
                    self.cpu = self.cpu.pin_memory()
                dptr = hip.host_device_pointer(self.cpu.data_ptr())
            else:
                # shm segments / file mappings: the rounded range is the mapping itself
                base = addr & ~(_PAGE - 1)
                size = -(-(addr + self.nbytes - base) // _PAGE) * _PAGE
                hip.host_register(base, size, True)
                self._reg_base = base
                dptr = hip.host_device_pointer(base) + (addr - base)
            self.rows = ops.HostRows(self.cpu, dptr)
            self.prep_stream = streams.batch_stream(self.device)
            # prep_streams = 2: consecutive batches' gathers alternate between two streams, so the next one
            # starts while the previous one's last workgroups drain (the link idles in a lone kernel's tail).
            # Not the default: two gathers in flight over the link were erratic on MI355X (16 workgroups:
            # 171-190k samples/s; 24-32: 20k-185k, profiles/r5_zerocopy/) against a steady 188k with one
            self._prep = [self.prep_stream] + [torch.cuda.Stream(self.device, priority=-1)
                                               for _ in range(max(1, int(prep_streams)) - 1)]
            self.prefault_s = self._prefault(dptr) if prefault else 0.0
        else:
            self.rows = self.cpu

    def _prefault(self, dptr: int) -> float:
        """Read one word of every 4 KB page of the mapped source once, before the first batch: the first
        pass of zero-copy gathers over never-touched mapped pages ran ~14% slower than every later pass
        (archive/profiles/r3_s2_final2). Returns the seconds it took (one small kernel, synchronised)."""
        import time

        if self.nbytes < 4:
            return 0.0
        t0 = time.perf_counter()
        blocks = 256
        sink = torch.empty(blocks, dtype=torch.int32, device=self.device)
        with streams.on_stream(self.prep_stream):
            _native.hip().touch_pages(dptr, self.nbytes, _PAGE, sink.data_ptr(), blocks,
                                      self.prep_stream.cuda_stream)
        self.prep_stream.synchronize()
        return time.perf_counter() - t0

    def _assemble(self, t: int):
        e, g = divmod(t, self.order.batches_per_epoch)
        kw = self._norm_kw()
        base = g * self.GB + self.rank * self.LB
        if self.prep_stream is None:
            return ops.gather_rows(self.rows, perm=self.order.perm(e), base=base, n_rows=self.LB,
                                   out_dtype=self.out_dtype, **kw), None
        st = self._prep[t % len(self._prep)]
        with streams.on_stream(st):
            out = self._out_batch((self.LB,) + self.sample_shape, self.out_dtype)
            batch = ops.gather_rows(self.rows, perm=self.order.perm(e), base=base, n_rows=self.LB, out=out,
                                    out_dtype=self.out_dtype, max_blocks=self.max_blocks, **kw)
            ev = torch.cuda.Event()
            ev.record(st)
        return batch, ev

    def stats(self) -> dict:
        return {"batches": self.batches, "source_bytes": self.nbytes, "max_blocks": self.max_blocks,
                "handoff": self.handoff, "host_waits": self.host_waits,
                "prefault_s": getattr(self, "prefault_s", 0.0),
                "prep_streams": len(self._prep) if self.prep_stream is not None else 0}

    def close(self) -> None:
        if self.prep_stream is not None:
            for st in self._prep:
                st.synchronize()
        self._queue.clear()
        self._blk, self._rec = None, [None, set()]
        if self._reg_base is not None:
            torch.cuda.synchronize(self.device)
            _native.hip().host_unregister(self._reg_base)
            self._reg_base = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
