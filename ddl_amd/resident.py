"""HBM-resident sharded dataset with an exact, world-size-invariant global shuffle.

BASELINE configs 3 and 5 ("datapusher scatter on RCCL over xGMI"; "global
shuffle across 8 ranks (on-device permute kernel) + prefetch-depth sweep at
288 GB HBM"). The reference can only trade a fraction of rows between the
k-th producers of two GPUs per window (reference ddl/shuffle.py:82-108), and
that code never runs. With 288 GB of HBM per MI355X a dataset
shard usually fits on the GPU, so here:

* the dataset (N samples) is sharded once across the W ranks -- rank r keeps
  rows [r*S, (r+1)*S) resident in HBM (S = ceil(N/W)), loaded through pinned
  bounce buffers on a copy stream;
* every epoch visits ``perm_e`` (the counter-based Feistel permutation of
  ``EpochOrder``): global batch g = perm_e(g*GB .. (g+1)*GB), rank r takes the
  slice [r*LB, (r+1)*LB) -- identical union for any W, so any rank may need
  any sample;
* batch assembly per step, on a prep stream, ``depth`` steps ahead:
  1. every rank knows the whole global batch (pure function of (seed, e, g)),
     so it knows which of ITS resident rows each peer needs -- no metadata is
     exchanged, only rows;
  2. the gfx950 ``gather_rows`` kernel packs the rows to send, grouped by
     destination;
  3. one RCCL ``all_to_all_single`` with per-peer split sizes over xGMI (all
     7 links of every GPU at once);
  4. a second ``gather_rows`` puts the received rows into batch order fused
     with the dtype cast and per-channel normalisation.
  With W = 1 step 4 alone runs, straight out of the resident shard, with the
  permutation evaluated inside the kernel.
* ``augment=`` replaces step 4 with the on-device RandomResizedCrop + flip +
  normalise kernel: an ImageNet-size uint8 dataset stays resident (193 GB at
  3x224x224) and every epoch sees fresh crops. The crop of a sample is keyed
  by (seed, epoch, global sample id), so it does not depend on W.

Checkpoint: the same ``kind="indexed"`` record as the loader
(seed, epoch, global_batch_cursor) -- resumable at any world size.
"""

from __future__ import annotations

import collections
import contextlib
import itertools
import math
import time
from typing import Any, Iterator

import numpy as np
import torch

from . import _native, ops
from .ops import _dtypes
from .parallel.order import check_group, issue, loader_group
from .permutation import EpochOrder, batch_cursor
from .types import DDLEnv
from .utils.logging import logger
from .utils import streams
from .utils.tracing import trace_range

STATE_VERSION = 1


def _source_address(source) -> tuple[int, int]:
    """(host address, rows) of a source: SharedArraySource / NpyMemmapSource / CPU tensor."""
    if isinstance(source, torch.Tensor):
        if source.is_cuda or not source.is_contiguous():
            raise ValueError("tensor sources must be contiguous CPU tensors")
        return source.data_ptr(), source.shape[0]
    if hasattr(source, "address"):
        return int(source.address), int(source.n)
    if hasattr(source, "_a"):
        a = source._a()
        return int(a.ctypes.data), int(source.n)
    raise TypeError(f"unsupported source {type(source).__name__}")


def _host_reader(source):
    """``read(row0, n_rows, dst_address, n_threads)`` copying rows [row0, row0+n) of a source
    into host memory: a parallel memcpy for in-memory sources, coalesced native
    ``pread`` for file-backed ones (``FileRowsSource``)."""
    if hasattr(source, "read_range"):
        return source.read_range
    addr, _ = _source_address(source)
    geom, dt = _source_geometry(source)
    row_bytes = (int(math.prod(geom)) if geom else 1) * _dtypes.itemsize(dt)
    rt = _native.runtime()

    def read(row0: int, n_rows: int, dst: int, n_threads: int) -> None:
        rt.parallel_copy(dst, addr + row0 * row_bytes, n_rows * row_bytes, n_threads)

    return read


def _source_rows(source) -> int:
    return int(source.n) if hasattr(source, "read_range") else _source_address(source)[1]


def _source_geometry(source) -> tuple[tuple[int, ...], torch.dtype]:
    if isinstance(source, torch.Tensor):
        return tuple(source.shape[1:]), source.dtype
    return tuple(source.sample_shape), _dtypes.to_torch_dtype(source.dtype)


class PrefetchedIndexedLoader:
    """Shared machinery of the device-assembled indexed loaders.

    Subclasses implement ``_assemble(t) -> (batch, ready_event)`` for global step
    ``t = epoch * batches_per_epoch + g``; this class runs it ``depth`` steps ahead
    (on the subclass's prep stream), hands each batch to the caller's stream and owns the
    ``kind="indexed"`` checkpoint cursor.

    Hand-off (``handoff``): "device" -- the caller's stream waits for the batch's ready event (a
    cross-queue barrier packet; the host never blocks); "host" -- the host waits for the event (usually
    already complete) and the caller's stream gets no barrier at all. A barrier packet costs the compute
    queue a ~30 us stall at every step boundary on MI355X when another queue is streaming (the zero-copy
    gather: step-boundary gaps 40 vs 10 us, GPU idle at r = 0.9 2.4% vs 0.7% on the producer path,
    ``profiles/r6_third``), so PCIe-paced loaders hand off on the host; loaders whose batches take
    microseconds keep the device hand-off by default, which never makes the host wait (behind a 1.25 ms step
    the HBM-resident loader idles 0.57% either way since batches come from blocks, ``profiles/r6_twentieth``;
    0.88-0.93% vs 0.81% before, ``profiles/r6_twelfth``; a host hand-off paces a host with no step of its own
    at the gather rate).
    """

    handoff = "device"
    block_bytes = 2 << 30  # output batches are carved from blocks of about this size (>= 1 batch, <= 64)

    def _out_batch(self, shape: tuple, dtype) -> torch.Tensor:
        """An output tensor for one batch, carved (on the current stream: the prep stream) from a block of
        batches. The caller's stream is recorded on a block once (``__iter__``), not once per batch: the caching
        allocator then puts one event on the compute stream when the block is freed, instead of one per batch
        -- each such event is a marker between two steps, and with the zero-copy gather streaming over PCIe a
        marker costs the compute queue ~14 us (step-boundary gap 32 -> 18 us, idle at r = 0.9 1.69 -> 0.97%
        without any, ``profiles/r6_nineteenth``). The batch engine's output slots do the same
        (``engine_dispatch._engine_provide``). A block is freed once every batch carved from it is gone."""
        n = int(math.prod(shape))
        blk = self._blk
        if blk is None or blk[0].dtype != dtype or blk[1] + n > blk[0].numel():
            per = max(1, min(64, self.block_bytes // max(1, n * torch.empty((), dtype=dtype).element_size())))
            blk = self._blk = [torch.empty(per * n, dtype=dtype, device=self.device), 0, set()]
            blk[2].add(streams.current(self.device.index).stream_id)  # the allocating stream
        cur = streams.current(self.device.index)
        if cur.stream_id not in blk[2]:  # another prep stream writes into this block: the allocator must know
            blk[0].record_stream(cur)
            blk[2].add(cur.stream_id)
        out = blk[0][blk[1]:blk[1] + n].view(shape)
        blk[1] += n
        return out

    def _record_caller(self, batch: torch.Tensor, cur) -> None:
        """``record_stream`` of the caller's stream on the batch's block (once per block and stream)."""
        base = batch._base if batch._base is not None else batch
        rec = self._rec
        if rec[0] is not base:
            rec = self._rec = [base, set()]
        if cur.stream_id not in rec[1]:
            base.record_stream(cur)
            rec[1].add(cur.stream_id)

    def _init_cursor(self, seed: int, depth: int, n_epochs: int | None, resume_state: dict | None) -> None:
        self.seed = int(seed)
        self.depth = max(1, int(depth))
        self.n_epochs = n_epochs
        self.epoch, self.cursor = 0, 0
        if resume_state is not None:
            self._apply_state(resume_state)
        self._pending = False
        self._queue: collections.deque = collections.deque()
        self._next_t = None
        self._generation = 0
        self.batches = 0
        self.host_waits = 0  # host hand-off: batches whose gather was still running when the caller asked
        self._blk = None  # [block tensor, elements carved] (_out_batch)
        self._rec = [None, set()]  # [block, caller streams recorded on it] (_record_caller)

    def __len__(self) -> int:
        """Batches left in the current epoch."""
        return self.order.batches_per_epoch - self.cursor

    @property
    def batches_per_epoch(self) -> int:
        return self.order.batches_per_epoch

    def _norm_kw(self) -> dict:
        norm = self.normalize
        if norm is None:
            return {}
        c = self.sample_shape[0] if len(self.sample_shape) > 1 else len(norm.get("mean", [0]))
        plane = int(math.prod(self.sample_shape[1:])) if len(self.sample_shape) > 1 else 1
        sc, bi = ops.norm_affine(c, norm.get("mean"), norm.get("std"), norm.get("scale"), norm.get("bias"),
                                 ops.pixel_max(self.src_dtype))
        return dict(scale=sc, bias=bi, plane=plane)

    def _total_steps(self) -> int | None:
        return None if self.n_epochs is None else self.n_epochs * self.order.batches_per_epoch

    def _fill(self, upto: int) -> None:
        total = self._total_steps()
        while self._next_t < upto and (total is None or self._next_t < total):
            self._queue.append((self._next_t,) + self._assemble(self._next_t))
            self._next_t += 1

    def __iter__(self) -> Iterator[torch.Tensor]:
        """One epoch of batches ([LB, *sample_shape] in ``out_dtype``)."""
        bpe = self.order.batches_per_epoch
        if self._pending:  # the previous iterator was left after yielding: that batch counts as consumed
            self._pending = False
            self.cursor += 1
            if self.cursor >= bpe:
                self.epoch, self.cursor = self.epoch + 1, 0
        self._generation += 1  # at most one live iterator: an older one stops at its next step
        gen = self._generation
        if self.n_epochs is not None and self.epoch >= self.n_epochs:
            return
        t0 = self.epoch * bpe + self.cursor
        if self._next_t is None:
            self._next_t = t0
        for t in range(t0, (self.epoch + 1) * bpe):
            if gen != self._generation:  # load_state_dict / set_epoch repositioned the loader
                return
            self._fill(t + self.depth)
            tq, batch, ev = self._queue.popleft()
            assert tq == t, (tq, t)
            if ev is not None:
                cur = streams.current(self.device.index)
                if self.handoff == "host":
                    if not ev.query():
                        self.host_waits += 1
                        ev.synchronize()  # a gather kernel of this process: it always completes
                else:
                    cur.wait_event(ev)
                self._record_caller(batch, cur)
            self.cursor = t - self.epoch * bpe
            self._pending = True
            self.batches += 1
            yield batch
            if gen != self._generation:
                return
            self._pending = False
            self.cursor += 1
        self.epoch += 1
        self.cursor = 0

    # ----------------------------------------------------------- checkpoint
    def state_dict(self) -> dict:
        return {
            "version": STATE_VERSION,
            "kind": "indexed",
            "seed": self.seed,
            "order_seed": self.seed,
            "epoch": self.epoch,
            "global_batch_cursor": self.cursor + (1 if self._pending else 0),
            # the same position in samples of the epoch order (the epoch/sample-index format)
            "global_sample_cursor": (self.cursor + (1 if self._pending else 0)) * self.order.global_batch,
            "batches_per_epoch": self.order.batches_per_epoch,
            "global_batch": self.order.global_batch,
            "n_samples": self.order.n_samples,
            "world_size": getattr(self, "W", 1),
            "dtype": str(self.out_dtype).replace("torch.", ""),
        }

    def _apply_state(self, sd: dict) -> None:
        if sd.get("kind") != "indexed" or sd.get("version") != STATE_VERSION:
            raise ValueError("not an indexed loader state")
        for key, mine in (("global_batch", self.order.global_batch), ("n_samples", self.order.n_samples),
                          ("order_seed", self.seed)):
            if sd.get(key) is not None and sd[key] != mine:
                raise ValueError(f"checkpoint {key}={sd[key]} does not match {mine}")
        self.epoch = int(sd["epoch"])
        self.cursor = batch_cursor(sd, self.order.global_batch)
        if self.cursor >= self.order.batches_per_epoch:
            self.epoch, self.cursor = self.epoch + 1, 0

    def _reset_queue(self) -> None:
        """Drop the prefetched batches (their assembly is drained first) and restart at the cursor."""
        prep = getattr(self, "prep_stream", None)
        if prep is not None:
            prep.synchronize()
        self._queue.clear()
        self._next_t = None
        self._pending = False
        self._generation += 1  # an iterator started before this point stops instead of yielding stale data

    def load_state_dict(self, sd: dict) -> None:
        """Restore a ``state_dict()`` on the live loader (any world size with the same global batch);
        the next ``iter()`` continues exactly after the checkpointed batch."""
        saved = (self.epoch, self.cursor)
        try:
            self._apply_state(sd)
        except Exception:
            self.epoch, self.cursor = saved
            raise
        self._reset_queue()

    def set_epoch(self, epoch: int) -> None:
        """torch-style: the next ``iter()`` yields epoch ``epoch`` from its first batch (no-op if already there)."""
        if int(epoch) == self.epoch and self.cursor == 0 and not self._pending:
            return
        self.epoch, self.cursor = int(epoch), 0
        self._reset_queue()



class ResidentGlobalLoader(PrefetchedIndexedLoader):
    def __init__(self, source, global_batch: int, env: DDLEnv | None = None, *, seed: int = 0,
                 drop_last: bool = True, out_dtype: Any = None, normalize: dict | None = None, depth: int = 2,
                 device: str | torch.device | None = None, n_epochs: int | None = None,
                 resume_state: dict | None = None, chunk_bytes: int = 256 << 20, host_threads: int = 8,
                 scatter_from: int | None = None, augment: dict | None = None, replicate: bool | str = "auto",
                 hbm_fraction: float = 0.8, handoff: str = "device"):
        import torch.distributed as dist

        if handoff not in ("host", "device"):
            raise ValueError("handoff must be 'host' or 'device'")
        self.handoff = handoff

        aug_keys = {"size", "scale", "ratio", "flip_p", "layout"}
        if augment is not None and not set(augment) <= aug_keys:
            raise ValueError(f"unknown augment keys {sorted(set(augment) - aug_keys)}")
        self.augment = augment

        self.env = env or DDLEnv()
        self.W, self.rank = self.env.world_size, self.env.rank
        self.scatter_from = scatter_from
        if scatter_from is not None and self.W > 1:
            # only `scatter_from` holds the dataset: broadcast its geometry (small metadata)
            geom = [None]
            if self.rank == scatter_from:
                shp, dt = _source_geometry(source)
                geom = [(shp, str(dt).replace("torch.", ""), _source_rows(source))]
            dist.broadcast_object_list(geom, src=scatter_from, group=self.env.control_group)
            shp, dt, n = geom[0]
            self.sample_shape, self.src_dtype = tuple(shp), _dtypes.to_torch_dtype(dt)
            reader = _host_reader(source) if self.rank == scatter_from else None
        else:
            self.sample_shape, self.src_dtype = _source_geometry(source)
            reader, n = _host_reader(source), _source_rows(source)
        self.row_elems = int(math.prod(self.sample_shape)) if self.sample_shape else 1
        self.row_bytes = self.row_elems * _dtypes.itemsize(self.src_dtype)
        self.N = n
        if not drop_last:  # the device-side order covers whole global batches only
            raise ValueError(f"{type(self).__name__} needs drop_last=True")
        self.order = EpochOrder(n, global_batch, seed, drop_last)
        self.GB = int(global_batch)
        self.LB = self.order.local_batch(self.W)
        self.S = -(-n // self.W)
        self.lo = self.rank * self.S
        self.hi = min(n, self.lo + self.S)
        if device is None:
            device = self.env.device or ("cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.out_dtype = _dtypes.to_torch_dtype(out_dtype) if out_dtype is not None else self.src_dtype
        self.normalize = normalize
        if augment is not None and (self.device.type != "cuda" or len(self.sample_shape) != 3):
            raise ValueError("augment= needs a GPU and [C, H, W] / [H, W, C] image samples")
        self._init_cursor(seed, depth, n_epochs, resume_state)
        self.group = None
        if self.W > 1:
            # the DP group: one communicator / RCCL stream with the trainer's DDP (parallel/order.py)
            self.group = loader_group(self.env)
        self.bytes_exchanged = 0
        self.bytes_replicated = 0
        self.replicated = self._decide_replicate(replicate, chunk_bytes, hbm_fraction)
        self.replicate_s = 0.0
        t0 = time.perf_counter()
        if self.replicated and self.W > 1:
            self.shard = self._load_replica(reader, chunk_bytes, host_threads, scatter_from)
        elif scatter_from is not None and self.W > 1:
            self.shard = self._scatter_shards(reader, chunk_bytes, host_threads, scatter_from)
        else:
            self.shard = self._load_shard(reader, chunk_bytes, host_threads)
        self.load_s = time.perf_counter() - t0
        self.resident_rows = int(self.shard.shape[0])
        self.prep_stream = streams.batch_stream(self.device) if self.device.type == "cuda" else None
        if self.device.type == "cuda" and self.W > 1 and not self.replicated:  # owner-bucketing outputs (prep stream)
            self._send_idx = torch.empty(self.GB, dtype=torch.int64, device=self.device)
            self._inv_idx = torch.empty(self.LB, dtype=torch.int64, device=self.device)

    # ----------------------------------------------------------------- load
    def _decide_replicate(self, replicate: bool | str, chunk_bytes: int, hbm_fraction: float) -> bool:
        """``replicate``: True / False, or "auto" = a whole replica (plus the bring-up's gather staging) fits in
        ``hbm_fraction`` of the free HBM of EVERY rank (MIN over the control group, so all ranks agree). At
        W = 1 the two layouts are the same (the rank's shard is the whole dataset): reported as replicated
        unless ``replicate=False``, loaded and stepped as one shard. "auto" on the CPU keeps the sharded layout
        at W > 1."""
        if replicate not in (True, False, "auto"):
            raise ValueError("replicate must be True, False or 'auto'")
        if self.W == 1:
            return replicate is not False
        if replicate != "auto":
            return bool(replicate)
        if self.device.type != "cuda":
            return False
        import torch.distributed as dist

        free, _ = torch.cuda.mem_get_info(self.device)
        need = self.S * self.W * self.row_bytes + self.W * self._chunk_rows(chunk_bytes) * self.row_bytes
        t = torch.tensor([1 if need <= hbm_fraction * free else 0], dtype=torch.int64)
        if self.env.control_group is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.env.control_group)
        logger.info("resident loader: replica %.1f GB vs %.1f GB free HBM -> %s", need / 1e9, free / 1e9,
                    "replicated" if t.item() else "sharded")
        return bool(t.item())

    def _chunk_rows(self, chunk_bytes: int) -> int:
        return max(1, min(self.S, chunk_bytes // max(self.row_bytes, 1)))

    def _load_replica(self, reader, chunk_bytes: int, host_threads: int, scatter_from: int | None) -> torch.Tensor:
        """The whole dataset resident on every rank, built without a host read of more than 1/W of it per rank.

        Each rank loads its slice [r*S, (r+1)*S) from the host exactly as the sharded mode does (pinned bounce
        buffers, PCIe, all ranks in parallel), straight into its place in the replica; then chunked RCCL
        ``all_gather``s over xGMI fill the other W-1 slices (chunk_bytes per rank per round: the collective's
        flat staging stays at W x chunk_bytes of HBM). With ``scatter_from`` only that rank holds the dataset:
        it streams chunks H2D and distributes each one as a scatter + all-gather -- grouped point-to-point
        sends of piece q of the chunk to rank q (every xGMI link of the source carries 1/W of the chunk at
        once), then an all-gather of the pieces -- instead of a ring broadcast, which is bound by one link
        (SURVEY §5, MI355X-native communication design). The replica has at least S*W rows (padding rows past
        N, never addressed: the epoch permutation ranges over [0, N)). Steps then gather the rank's slice of
        every global batch from its own replica: no per-step collective at all."""
        import torch.distributed as dist

        W = self.W
        rows_total = max(self.S * W, self.N + W)  # + the last scatter chunk's piece padding
        replica = torch.empty((rows_total,) + self.sample_shape, dtype=self.src_dtype, device=self.device)
        probe = torch.zeros(1, device=self.device)
        issue(self.env, self.group, "resident.bringup")
        dist.all_reduce(probe, group=self.group)  # communicator bring-up on every rank before the timed parts
        cr = self._chunk_rows(chunk_bytes)
        if scatter_from is None:
            self._load_rows(reader, replica, self.lo, self.hi - self.lo, chunk_bytes, host_threads)
            t0 = time.perf_counter()
            with trace_range("ddl.resident.replicate"):
                for k, c0 in enumerate(range(0, self.S, cr)):
                    c1 = min(self.S, c0 + cr)
                    outs = [replica[q * self.S + c0:q * self.S + c1] for q in range(W)]
                    issue(self.env, self.group, "resident.replicate", k)
                    dist.all_gather(outs, outs[self.rank], group=self.group)
                    self.bytes_replicated += (W - 1) * (c1 - c0) * self.row_bytes
        else:
            t0 = time.perf_counter()
            src = self.rank == scatter_from
            span = W * max(1, -(-cr // W))  # chunk rows: W pieces
            with trace_range("ddl.resident.replicate"):
                for k, c0 in enumerate(range(0, self.N, span)):
                    n_rows = min(span, self.N - c0)
                    pr = -(-n_rows // W)  # piece rows (the last piece may run into the padding)
                    pieces = [replica[c0 + q * pr:c0 + (q + 1) * pr] for q in range(W)]
                    if src:
                        self._load_rows(reader, replica, c0, n_rows, chunk_bytes, host_threads)
                        p2p = [dist.P2POp(dist.isend, pieces[q], q, group=self.group) for q in range(W)
                               if q != scatter_from]
                    else:
                        p2p = [dist.P2POp(dist.irecv, pieces[self.rank], scatter_from, group=self.group)]
                    check_group(self.env, self.group, "resident.replicate_scatter")
                    for req in dist.batch_isend_irecv(p2p):
                        req.wait()
                    issue(self.env, self.group, "resident.replicate", k)
                    dist.all_gather(pieces, pieces[self.rank], group=self.group)
                    self.bytes_replicated += (W - 1) * pr * self.row_bytes * (2 if src else 1)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.replicate_s = time.perf_counter() - t0
        return replica

    def _load_rows(self, reader, dst: torch.Tensor, row0: int, rows: int, chunk_bytes: int,
                   host_threads: int) -> None:
        """Source rows [row0, row0 + rows) into ``dst[row0:row0 + rows]`` (device or host tensor)."""
        if rows <= 0:
            return
        out = dst[row0:row0 + rows].view(-1).view(torch.uint8)
        if self.device.type != "cuda":
            reader(row0, rows, out.data_ptr(), host_threads)
            return
        self._h2d_rows(reader, out, row0, rows, chunk_bytes, host_threads)

    def _load_shard(self, reader, chunk_bytes: int, host_threads: int) -> torch.Tensor:
        rows = self.hi - self.lo
        shard = torch.empty((rows,) + self.sample_shape, dtype=self.src_dtype, device=self.device)
        if rows == 0:
            return shard
        dst_bytes = shard.view(-1).view(torch.uint8)
        if self.device.type != "cuda":
            reader(self.lo, rows, dst_bytes.data_ptr(), host_threads)
            return shard
        self._h2d_rows(reader, dst_bytes, self.lo, rows, chunk_bytes, host_threads)
        return shard

    def _h2d_rows(self, reader, dst_bytes: torch.Tensor, row0: int, rows: int, chunk_bytes: int,
                  host_threads: int) -> None:
        """Source rows [row0, row0 + rows) into the HBM bytes ``dst_bytes``: double-buffered pinned bounce
        buffers, host read (memcpy / pread) || SDMA H2D."""
        hip = _native.hip()
        chunk_rows = max(1, min(chunk_bytes // max(self.row_bytes, 1), rows))
        bufs = [torch.empty(chunk_rows * self.row_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        evs = [torch.cuda.Event(), torch.cuda.Event()]
        used = [False, False]
        s = torch.cuda.Stream(self.device)
        r, i = 0, 0
        with trace_range("ddl.resident.load"):
            while r < rows:
                n = min(chunk_rows, rows - r)
                b = i % 2
                if used[b]:
                    evs[b].synchronize()
                reader(row0 + r, n, bufs[b].data_ptr(), host_threads)
                hip.memcpy_h2d(dst_bytes.data_ptr() + r * self.row_bytes, bufs[b].data_ptr(), n * self.row_bytes,
                               s.cuda_stream)
                evs[b].record(s)
                used[b] = True
                r += n
                i += 1
            s.synchronize()

    def _scatter_shards(self, reader, chunk_bytes: int, host_threads: int, src_rank: int) -> torch.Tensor:
        """Rank ``src_rank`` streams the dataset H2D chunk by chunk and sends every
        peer the rows of its shard with grouped point-to-point ops (all peers at
        once: on an xGMI-connected node every link carries one peer's slice);
        the other ranks receive straight into their HBM shard.

        Pipelined on the source rank, double-buffered, with no per-chunk stream
        synchronisation: while the host reads chunk i+1 into pinned bounce buffer
        b', the copy stream moves chunk i bounce[b] -> HBM staging[b] and the send
        stream ships staging[b]'s slices over RCCL. The host blocks only before
        re-filling a bounce buffer (its previous H2D must have retired); the copy
        stream waits before re-filling a staging buffer (its previous sends must
        have completed): read || H2D || P2P.
        """
        import torch.distributed as dist

        rows = self.hi - self.lo
        shard = torch.empty((rows,) + self.sample_shape, dtype=self.src_dtype, device=self.device)
        # first op on the group must be collective (communicator bring-up on every rank)
        probe = torch.zeros(1, device=self.device)
        issue(self.env, self.group, "resident.bringup")
        dist.all_reduce(probe, group=self.group)
        rows_per_chunk = max(1, chunk_bytes // self.row_bytes)
        bounds = [(q * self.S, min(self.N, (q + 1) * self.S)) for q in range(self.W)]
        gpu = self.device.type == "cuda"
        src = self.rank == src_rank
        if src:
            staging = [torch.empty((rows_per_chunk,) + self.sample_shape, dtype=self.src_dtype, device=self.device)
                       for _ in range(2)]
            bounce = [torch.empty(rows_per_chunk * self.row_bytes, dtype=torch.uint8, pin_memory=gpu)
                      for _ in range(2)]
            if gpu:
                copy_s, send_s = torch.cuda.Stream(self.device), torch.cuda.Stream(self.device)
                h2d_done = [torch.cuda.Event(), torch.cuda.Event()]
                sent = [torch.cuda.Event(), torch.cuda.Event()]
                used = [False, False]
        with trace_range("ddl.resident.scatter"):
            for i, c0 in enumerate(range(0, self.N, rows_per_chunk)):
                c1 = min(self.N, c0 + rows_per_chunk)
                ops_ = []
                if src:
                    b = i % 2
                    nbytes = (c1 - c0) * self.row_bytes
                    if gpu and used[b]:
                        h2d_done[b].synchronize()  # bounce[b]'s previous H2D retired
                    reader(c0, c1 - c0, bounce[b].data_ptr(), host_threads)
                    stage = staging[b][: c1 - c0]
                    if gpu:
                        if used[b]:
                            copy_s.wait_event(sent[b])  # staging[b]'s previous sends completed
                        with streams.on_stream(copy_s):
                            stage.view(-1).view(torch.uint8)[:nbytes].copy_(bounce[b][:nbytes], non_blocking=True)
                        h2d_done[b].record(copy_s)
                        send_s.wait_event(h2d_done[b])
                        used[b] = True
                    else:
                        stage.view(-1).view(torch.uint8)[:nbytes].copy_(bounce[b][:nbytes])
                    ctx = streams.on_stream(send_s) if gpu else contextlib.nullcontext()
                    with ctx:
                        for q, (lo, hi) in enumerate(bounds):
                            o0, o1 = max(c0, lo), min(c1, hi)
                            if o0 >= o1:
                                continue
                            piece = stage[o0 - c0:o1 - c0]
                            if q == self.rank:
                                shard[o0 - lo:o1 - lo].copy_(piece)
                            else:
                                ops_.append(dist.P2POp(dist.isend, piece, q, group=self.group))
                        self.bytes_exchanged += sum(p.tensor.numel() * p.tensor.element_size() for p in ops_)
                        if ops_:  # point-to-point (pairwise), not a collective: no ledger entry
                            check_group(self.env, self.group, "resident.scatter_p2p")
                            for req in dist.batch_isend_irecv(ops_):
                                req.wait()  # the send stream (not the host) waits for the sends
                        if gpu:
                            sent[b].record(send_s)
                else:
                    o0, o1 = max(c0, self.lo), min(c1, self.hi)
                    if o0 < o1:
                        ops_.append(dist.P2POp(dist.irecv, shard[o0 - self.lo:o1 - self.lo], src_rank,
                                               group=self.group))
                        check_group(self.env, self.group, "resident.scatter_p2p")
                        for req in dist.batch_isend_irecv(ops_):
                            req.wait()
        if gpu:
            torch.cuda.synchronize(self.device)
        return shard

    def _assemble(self, t: int) -> tuple[torch.Tensor, Any]:
        """Enqueue the assembly of global step t = epoch*bpe + g; returns (batch, ready event)."""
        import torch.distributed as dist

        if self.shard is None:
            raise RuntimeError("ResidentGlobalLoader is closed (its HBM shard was released)")
        e, g = divmod(t, self.order.batches_per_epoch)
        perm = self.order.perm(e)
        kw = self._norm_kw()
        ctx = streams.on_stream(self.prep_stream) if self.prep_stream is not None else contextlib.nullcontext()
        with ctx, trace_range("ddl.resident.assemble"):
            if self.W == 1 or self.replicated:
                # the resident rows ARE global sample ids (W = 1, or a whole replica): the rank's slice of
                # global batch g straight from HBM, the permutation evaluated inside the kernel
                base = g * self.GB + self.rank * self.LB
                if self.augment is not None:
                    batch = self._crop(self.shard, e, perm=perm, base=base, n_rows=self.LB)
                else:
                    out = self._out_batch((self.LB,) + self.sample_shape, self.out_dtype) \
                        if self.prep_stream is not None else None
                    batch = ops.gather_rows(self.shard, perm=perm, base=base, n_rows=self.LB, out=out,
                                            out_dtype=self.out_dtype, **kw)
            else:
                # W split counts on the host (native Feistel over the GB positions, no numpy); the send list
                # and the receive map by the owner-bucketing kernels on the prep stream (csrc/kernels/bucket.hip)
                pos0 = g * self.GB
                mine0 = pos0 + self.rank * self.LB
                send_counts, recv_counts = _native.runtime().owner_counts(
                    perm.keys, perm.half_bits, self.N, pos0, self.GB, self.LB, self.S, self.W, self.rank)
                n_send = sum(send_counts)
                if self.device.type == "cuda":
                    hip, stream = _native.hip(), self.prep_stream.cuda_stream
                    hip.bucket_send(perm.keys, self.N, perm.half_bits, pos0, self.GB, self.S, self.lo, self.rank,
                                    self.W, self._send_idx.data_ptr(), stream)
                    offsets = [0, *itertools.accumulate(recv_counts[:-1])]
                    hip.bucket_recv(perm.keys, self.N, perm.half_bits, mine0, self.LB, self.S, self.W, offsets,
                                    self._inv_idx.data_ptr(), stream)
                    send_idx, inv = self._send_idx[:n_send], self._inv_idx
                else:  # CPU rehearsal: the same maps from the native host twin of the kernels
                    s_np, i_np = _native.runtime().owner_maps(perm.keys, perm.half_bits, self.N, pos0, self.GB,
                                                              self.LB, self.S, self.W, self.rank, self.lo)
                    send_idx, inv = torch.from_numpy(s_np), torch.from_numpy(i_np)
                send = ops.gather_rows(self.shard, index=send_idx) if n_send else \
                    torch.empty((0,) + self.sample_shape, dtype=self.src_dtype, device=self.device)
                recv = torch.empty((self.LB,) + self.sample_shape, dtype=self.src_dtype, device=self.device)
                issue(self.env, self.group, "resident.all_to_all", t)
                dist.all_to_all_single(recv.view(self.LB, -1), send.view(send.shape[0], -1), recv_counts,
                                       send_counts, group=self.group)
                self.bytes_exchanged += (n_send - send_counts[self.rank]) * self.row_bytes
                if self.augment is not None:  # crop keyed by the global sample id, not the recv row
                    ids = ops.feistel_indices(perm, mine0, self.LB, device=self.device) \
                        if self.device.type == "cuda" else torch.from_numpy(perm(np.arange(mine0, mine0 + self.LB)))
                    batch = self._crop(recv, e, index=inv, sample_ids=ids)
                else:
                    batch = ops.gather_rows(recv, index=inv, out_dtype=self.out_dtype, **kw)
            ev = None
            if self.prep_stream is not None:
                ev = torch.cuda.Event()
                ev.record(self.prep_stream)
        return batch, ev

    def _crop(self, src: torch.Tensor, epoch: int, **kw) -> torch.Tensor:
        from .batching import _mix

        aug, norm = self.augment, self.normalize or {}
        return ops.random_resized_crop(
            src, size=aug.get("size", (224, 224)), scale=aug.get("scale", (0.08, 1.0)),
            ratio=aug.get("ratio", (3.0 / 4.0, 4.0 / 3.0)), flip_p=aug.get("flip_p", 0.5),
            seed=_mix(self.seed, epoch), layout=aug.get("layout", "chw"),
            out_dtype=self.out_dtype if self.out_dtype in (torch.bfloat16, torch.float32) else torch.bfloat16,
            mean=norm.get("mean"), std=norm.get("std"), **kw)

    def stats(self) -> dict:
        rows = self.resident_rows
        return {"batches": self.batches, "replicated": self.replicated, "bytes_exchanged": self.bytes_exchanged,
                "bytes_replicated": self.bytes_replicated, "resident_rows": rows,
                "shard_rows": self.hi - self.lo, "shard_bytes": rows * self.row_bytes,
                "load_s": self.load_s, "replicate_s": self.replicate_s}

    def close(self) -> None:
        """Drain the prep stream and release the HBM shard (a 150-190 GB shard must be
        gone before the next loader allocates its own, even while a generator still
        references this object)."""
        if self.prep_stream is not None:
            self.prep_stream.synchronize()
        self._queue.clear()
        self._blk, self._rec = None, [None, set()]
        logger.debug("resident loader closed: %s", self.stats())
        self.shard = None

