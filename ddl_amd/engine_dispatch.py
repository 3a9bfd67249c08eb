"""Native per-batch dispatch of ``DistributedDataLoader`` (the C++ ``BatchEngine``, csrc/kernels/engine.cpp).

The reference slices its batch out of the shared window on the host
(``/root/reference/ddl/mpi_dataloader.py:179-198``). Here a batch is a gfx950 kernel launch over the
staged HBM window (Feistel gather + cast / normalise, HWC -> CHW collate, a contiguous column split, or a
token pad/pack),
and the engine issues it from C++: inline on the caller's stream, one launch per window, or one batch
ahead on the high-priority batch stream. The Python dispatch path (``native_dispatch=False``) builds the
same batches with the same kernels; it serves the two recipes the engine does not (on-device augment, and
zero-copy split views of the window) and is the engine's test oracle.
"""

from __future__ import annotations

import math
import os

import torch

from . import ops
from .ops import _dtypes
from .utils import streams
from .utils.tracing import trace_range

_TRACE_ENGINE = os.environ.get("DDL_ROCTX", "1") == "2"  # roctx level 2: also a range per native get


class NativeDispatchMixin:
    """Recipe selection, engine construction, output-slot blocks and the per-batch ``get``."""

    # output slots come from blocks of about this size (4..128 slots): the caching allocator puts one event on
    # the consumer's stream per freed block, a marker between two steps (~10 us of step-boundary gap). 2 GB:
    # 26 slots of 77 MB per event, GPU idle at r = 0.9 0.77-0.80% -> 0.70-0.71% vs 512 MB
    # (profiles/r6_twentythird); two blocks are allocated up front, 4 GB of the 288 GB HBM
    engine_block_bytes = 2 << 30

    def _engine_recipe(self) -> dict | None:
        """The batch recipe when the native engine can build batches exactly like ``_batch_from_window``:
        a fused gather (one output), a contiguous column split or a token pad/pack; no HWC collate or
        augment. The global-shuffle exchange is compatible: it rewrites the staged window in place on the
        post-copy stream before the window's ready event, which is what the engine's launches wait on
        (``_ensure_posted`` issues it before the engine touches the window)."""
        if not self.native_dispatch or self._batch_stream is None:
            return None
        if self.collate == "tokens":
            return self._token_recipe()
        if self.augment is not None:
            return self._augment_recipe()
        if self.collate is not None:
            return None
        norm = self.normalize
        wdt = self.window_dtype
        if norm is not None and norm.get("layout", "chw") == "hwc":
            return self._hwc_recipe(norm, wdt)
        out_dtype = self.out_dtype or (torch.float32 if norm is not None else wdt)
        splits = list(self.splits[0])
        rec = dict(in_dt=_dtypes.code(wdt), out_dt=_dtypes.code(out_dtype), shuffle=self.shuffle == "device",
                   batch=self.batch_size, seed=self.seed & ((1 << 64) - 1), max_blocks=0, scale=[],
                   bias=[],
                   plane=0, n_data=[int(x.nData) for x in self.metadata_from_producer], widths=[])
        if (self.contiguous or self.copy_batches) and len(splits) > 1 and len(self.sample_shape) == 1 \
                and norm is None:
            if out_dtype != wdt and out_dtype not in (torch.bfloat16, torch.float32):
                return None
            rec.update(kind=1, row_elems=int(self.sample_shape[0]), widths=[int(w) for w in splits],
                       out_shapes=[(self.batch_size, int(w)) for w in splits], out_dtype=out_dtype)
            return rec
        if len(splits) != 1:
            return None  # gather + split views: Python path
        if self.shuffle != "device" and out_dtype == wdt and norm is None and not self.copy_batches:
            return None  # zero-copy view of the window
        if out_dtype != wdt and (out_dtype not in (torch.bfloat16, torch.float16, torch.float32)
                                 or wdt not in (torch.uint8, torch.float32, torch.bfloat16, torch.float16)):
            return None  # a conversion the gather kernel does not do: the Python path reports it
        if norm is not None:
            plane = int(math.prod(self.sample_shape[1:])) if len(self.sample_shape) > 1 else 1
            c = self.sample_shape[0] if len(self.sample_shape) > 1 else len(norm.get("mean", [0]))
            sc, bi = ops.norm_affine(c, norm.get("mean"), norm.get("std"), norm.get("scale"), norm.get("bias"),
                                     ops.pixel_max(wdt))
            if out_dtype in (torch.uint8, torch.int32, torch.int64):
                return None
            rec.update(scale=[float(x) for x in sc], bias=[float(x) for x in bi], plane=plane)
        rec.update(kind=0, row_elems=int(math.prod(self.sample_shape)) if self.sample_shape else 1,
                   out_shapes=[(self.batch_size,) + tuple(self.sample_shape)], out_dtype=out_dtype)
        return rec

    def _augment_recipe(self) -> dict | None:
        """On-device RandomResizedCrop + flip + normalise + cast (csrc/kernels/augment.hip) launched by the engine.
        Crops are keyed exactly as on the Python path: (seed mixed with the window's epoch, producer, producer
        round, source row); the engine derives the epoch from the window index (``set_epoch_base``)."""
        aug, norm = self.augment, self.normalize or {}
        shape, wdt = tuple(self.sample_shape), self.window_dtype
        layout = aug.get("layout", "chw")
        out_dtype = self.out_dtype or torch.bfloat16
        if (len(shape) != 3 or len(self.splits[0]) != 1 or out_dtype not in (torch.bfloat16, torch.float32)
                or wdt not in (torch.uint8, torch.float32, torch.bfloat16)):
            return None
        c, h, w = (shape[2], shape[0], shape[1]) if layout == "hwc" else shape
        oh, ow = aug.get("size", (224, 224))
        sc, bi = ops.norm_affine(int(c), norm.get("mean"), norm.get("std"), None, None, ops.pixel_max(wdt))
        scale, ratio = aug.get("scale", (0.08, 1.0)), aug.get("ratio", (3.0 / 4.0, 4.0 / 3.0))
        return dict(kind=4, in_dt=_dtypes.code(wdt), out_dt=_dtypes.code(out_dtype), shuffle=self.shuffle == "device",
                    batch=self.batch_size, seed=self.seed & ((1 << 64) - 1), max_blocks=0,
                    scale=[float(x) for x in sc], bias=[float(x) for x in bi], plane=1,
                    n_data=[int(x.nData) for x in self.metadata_from_producer], widths=[],
                    row_elems=int(math.prod(shape)), aug_seed=self.seed & ((1 << 64) - 1),
                    augment=[1.0 if layout == "hwc" else 0.0, float(h), float(w), float(c), float(oh), float(ow),
                             float(scale[0]), float(scale[1]), float(ratio[0]), float(ratio[1]),
                             float(aug.get("flip_p", 0.5))],
                    outputs=[((self.batch_size, int(c), int(oh), int(ow)), out_dtype),
                             ((self.batch_size, 5), torch.int32)],
                    augment_outputs=True)

    def _hwc_recipe(self, norm: dict, wdt) -> dict | None:
        """HWC image rows ([H, W, C], e.g. decoded JPEGs) -> normalised CHW batches: the LDS-tiled collate kernel
        (csrc/kernels/collate.hip) launched by the engine, like the gather."""
        shape = tuple(self.sample_shape)
        out_dtype = self.out_dtype or torch.float32
        if (len(shape) < 2 or len(self.splits[0]) != 1 or out_dtype not in (torch.bfloat16, torch.float32)
                or wdt not in (torch.uint8, torch.float32, torch.bfloat16)):
            return None
        c, pixels = int(shape[-1]), int(math.prod(shape[:-1]))
        sc, bi = ops.norm_affine(c, norm.get("mean"), norm.get("std"), norm.get("scale"), norm.get("bias"),
                                 ops.pixel_max(wdt))
        return dict(kind=3, in_dt=_dtypes.code(wdt), out_dt=_dtypes.code(out_dtype), shuffle=self.shuffle == "device",
                    batch=self.batch_size, seed=self.seed & ((1 << 64) - 1), max_blocks=0,
                    scale=[float(x) for x in sc], bias=[float(x) for x in bi], plane=pixels,
                    n_data=[int(x.nData) for x in self.metadata_from_producer], widths=[c],
                    row_elems=c * pixels, out_shapes=[(self.batch_size, c) + shape[:-1]], out_dtype=out_dtype)

    def _token_recipe(self) -> dict | None:
        """Token windows (models/tokens.py): the pad/pack kernel straight from the staged window."""
        from .models.tokens import TokenWindowLayout

        ex = [m.extra for m in self.metadata_from_producer]
        if any(e.get("token_layout") != ex[0].get("token_layout") or e.get("token_mode") != ex[0].get("token_mode")
               for e in ex):
            return None
        lay = TokenWindowLayout(**ex[0]["token_layout"])
        mode = ex[0]["token_mode"]
        reg = lay.regions()
        S = lay.seq_len
        rows = lay.batch if mode == "pad" else lay.max_segments
        outs = [((rows, S), torch.int32), ((rows, S), torch.uint8), ((rows, S), torch.int64)]
        if mode == "pack":
            outs += [((rows, S), torch.int32), ((lay.max_segments + 1,), torch.int32)]
        fill = lay.max_segments if (mode == "pack" and self.token_rows == "fixed") else 0
        token = [0 if mode == "pad" else 1, int(self.pad_id), S, reg["offsets"][0], reg["row_start"][0],
                 reg["row_end"][0], reg["seg_offsets"][0], reg["tokens"][0], lay.header_stride, fill, lay.token_bytes]
        return dict(kind=2, in_dt=_dtypes.code(torch.int32), out_dt=_dtypes.code(torch.int32), shuffle=False,
                    batch=lay.batch, row_elems=1, seed=0, max_blocks=0, scale=[], bias=[], plane=0,
                    n_data=[int(x.nData) for x in self.metadata_from_producer], widths=[], token=token,
                    outputs=outs, token_mode=mode)

    def _make_engine(self) -> None:
        rec = self._engine_recipe()
        if rec is None:
            self._engine = None
            return
        import collections

        from . import _native

        st = self._stager
        if "outputs" in rec:
            self._eng_outputs = rec.pop("outputs")
        else:
            dt = rec.pop("out_dtype")
            self._eng_outputs = [(sh, dt) for sh in rec.pop("out_shapes")]
        self._eng_tokens = rec.pop("token_mode", None)
        self._eng_aug = rec.pop("augment_outputs", False)  # (images,) to the caller; the boxes stay in the slot
        self._engine = _native.hip().BatchEngine(
            st._native, n_producers=self.connection.n_producers, buffers=[b.data_ptr() for b in st.buffers],
            ready=[e.cuda_event for e in st.ready_events], batch_stream=self._batch_stream.cuda_stream,
            device=self.device.index, **rec)
        if self._eng_aug:
            self._engine.set_epoch_base(self.window - self.window_in_epoch, self.epoch, self.windows_per_epoch)
        # byte layout of one slot: every output 256-byte aligned, in order (a block holds K slots back to back)
        self._eng_layout, size = [], 0
        for sh, dt in self._eng_outputs:
            self._eng_layout.append((sh, dt, size))
            size += -(-math.prod(sh) * _dtypes.itemsize(dt) // 256) * 256
        self._eng_slot_bytes = max(256, size)
        self._eng_block = int(min(128, max(4, self.engine_block_bytes // self._eng_slot_bytes)))
        mode = self.native_dispatch
        bpw_max = max(self.batches_per_window)
        # whole-window launches: every window holds >= 2 batches, and consecutive slots of a block are one
        # contiguous run per output where the kernel needs that (gather: no slot padding; split takes a slot
        # stride; token windows get one pad/pack launch with a grid row per sub-batch)
        whole_ok = (min(self.batches_per_window) > 1 and rec["kind"] != 4  # augment: one launch per batch
                    and (rec["kind"] not in (0, 3) or self._eng_slot_bytes == math.prod(self._eng_outputs[0][0])
                         * _dtypes.itemsize(self._eng_outputs[0][1])))
        if mode == "auto":
            # small batches are host-bound: inline (no batch events, ~3 us of C++ per batch), or one launch per
            # window when a window holds several small batches; a large batch kernel (25 us for 256 images) is
            # worth overlapping with the previous step on the batch stream (GPU idle behind a train step 0.17%
            # lookahead vs 0.71% inline, archive/profiles/r2_native_dispatch)
            mode = "inline" if self._eng_slot_bytes < (16 << 20) else "lookahead"
            if mode == "inline" and whole_ok and self._eng_slot_bytes * bpw_max <= (256 << 20):
                mode = "window"
        if mode == "window" and not whole_ok:
            mode = "inline"
        self._eng_whole = mode == "window"
        if self._eng_whole:
            self._eng_block = max(self._eng_block, bpw_max)  # a window's slots come from one block
            self._engine.set_window_mode(True, self._eng_slot_bytes)
        self._engine.inline = mode in ("inline", "window")
        self._engine.set_batches_per_window([int(b) for b in self.batches_per_window])
        # a window's ring buffer goes back to the stager at its last batch launch, one step before the
        # consumer's release (archive/profiles/r3_early_release); a later out-of-order fetch of that window raises
        self._engine.early_release = True
        # lookahead batches still pending at get(): the host waits for them (no device-side cross-queue
        # barrier on the compute stream, archive/profiles/r3_handoff) -- also with the exchange on (round 6: GPU
        # idle at r = 0.9 through a 1-rank RCCL group 1.12-1.21% -> 0.84-0.85%, profiles/r6_tenth). The batch
        # kernel then waits on the exchange, a collective every rank issued at an EARLIER point of the schedule
        # (entering the previous window, parallel/order.py), so this host wait never closes a cycle across ranks;
        # a dead or hung peer ends it through the job abort / the process group's timeout
        self._engine.host_handoff = True
        # the host (not the batch stream) waits for a window's H2D copy before launching its batch kernels
        # (bounded by the loader timeout), so no queue holds a barrier packet on an unfinished copy: GPU idle
        # below the crossover 2.4-2.5% -> 1.1% at r = 0.9 (archive/profiles/r4_sixteenth, r4_seventeenth). Not
        # with the exchange, whose readiness is the post-copy stage's ready event (below)
        self._engine.ready_on_host = self._exchange_fn is None
        # with the exchange the window is ready when its post-copy stage's ready event completes: the host waits
        # for that event before the window's first launch, so the batch stream's queue holds no barrier packet on
        # a collective (GPU idle at r = 0.9 through a 1-rank RCCL group 0.84% -> 0.74-0.78%, profiles/r6_thirteenth)
        self._engine.ready_event_on_host = self._exchange_fn is not None
        # then the copy's retire event is the only marker behind it in the copy stream's queue
        self._stager._native.record_ready = not self._engine.ready_on_host
        self._eng_mode = mode
        self._eng_slots: collections.deque = collections.deque()  # (slot id, outputs, block)
        self._eng_next_id = 0
        self._eng_rec = (None, None)  # (block, stream) of the last record_stream
        self._eng_window = None
        self._eng_given: dict = {}  # local batch -> (outputs, block, tags) of the current window (re-fetch)
        self._eng_spare: dict = {}  # whole-window mode: slot id -> (outputs, block) built but not yet fetched
        self._eng_streams: dict = {}  # torch stream id -> (Stream, raw hipStream_t)
        self._eng_budget = 0
        # the first blocks are allocated up front, outside any timed loop: >= 24 slots, so that in steady
        # state every new block reuses a freed one from the caching allocator (no hipMalloc per block)
        for _ in range(max(2, -(-24 // self._eng_block))):
            self._engine_provide()

    def _engine_provide(self) -> None:
        """One allocation (on the batch stream) for a block of output slots; each slot is used once.
        The K slots' views of an output come from ONE strided view + ``unbind`` (per-slot slicing cost
        ~9 us per batch of host time on the box: three tensor ops per output per slot)."""
        K = self._eng_block
        with streams.on_stream(self._batch_stream), trace_range("ddl.engine.provide"):
            block = torch.empty(K * self._eng_slot_bytes, dtype=torch.uint8, device=self.device)
        base, sb, per_group, ptrs = block.data_ptr(), self._eng_slot_bytes, [], [[] for _ in range(K)]
        for sh, dt, off in self._eng_layout:
            isz = _dtypes.itemsize(dt)
            inner = [1] * len(sh)
            for d in range(len(sh) - 2, -1, -1):
                inner[d] = inner[d + 1] * sh[d + 1]
            per_group.append(block[off:].view(dt).as_strided((K,) + tuple(sh), (sb // isz,) + tuple(inner)).unbind(0))
            for k in range(K):
                ptrs[k].append(base + k * sb + off)
        first = self._eng_next_id
        self._eng_slots.extend(zip(range(first, first + K), zip(*per_group), [block] * K))
        self._eng_next_id += K
        self._engine.provide(ptrs)

    def _engine_raise(self, code: int, producer: int, what: str) -> None:
        from .exceptions import DDLError, DDLTimeoutError, PeerDeathError, ShutdownError

        if code <= -10:
            rc = -code - 10
            if rc == 1:
                raise ShutdownError(f"{what}: loader was shut down")
            if rc == 2:
                raise DDLTimeoutError(f"{what}: not staged within {self.timeout_s:.0f}s (producer {producer})")
            pids = self.connection.producer_pids
            pid = pids[producer] if 0 <= producer < len(pids) else None
            if rc in (3, 4):
                raise PeerDeathError(f"{what}: producer {producer} (pid {pid}) "
                                     + ("reported a failure" if rc == 4 else "died"), producer, pid)
            raise DDLError(f"{what}: {self._stager._native.error()}")
        if code == -4:  # the host wait for the window's H2D copy failed (the stager's error names it)
            err = self._stager._native.error() or "waiting for the window's H2D copy failed"
            raise (DDLTimeoutError if self._stager._native.error_code == 2 else DDLError)(f"{what}: {err}")
        if code == -3:
            raise DDLError(f"{what}: requested out of order after the window's last batch -- a window goes back "
                           "to the prefetcher when its last batch is launched; within a window, fetch batches "
                           "in order (a batch already fetched can be fetched again)")
        raise DDLError(f"{what}: native batch engine error {code}")

    def _engine_batch(self, local: int, bpw: int):
        eng = self._engine
        if self._eng_whole:
            if local == 0:  # the window's bpw slots, after at most the skipped tail of a block
                while eng.slots_left < bpw + self._eng_block:
                    self._engine_provide()
        else:
            self._eng_budget -= 2  # a get takes at most 2 slots (the batch + a lookahead): query only when low
            if self._eng_budget < 4:
                if eng.slots_left < 4:
                    self._engine_provide()
                self._eng_budget = eng.slots_left
        sid = torch._C._cuda_getCurrentStream(self.device.index)
        hit = self._eng_streams.get(sid)
        if hit is None:
            st = streams.current(self.device.index)
            hit = self._eng_streams[sid] = (st, st.cuda_stream)
        cur, handle = hit
        w = self.window
        if self._eng_window == w:
            again = self._eng_given.get(local)
            if again is not None:  # fetched before in this window: the same outputs (slots are used once)
                out, block, tags = again
                if self._eng_rec[0] is not block or self._eng_rec[1] is not cur:
                    block.record_stream(cur)
                    self._eng_rec = (block, cur)
                return self._engine_outputs(out, tags)
        nxt = self.window_in_epoch + 1 < self.windows_per_epoch or self.epoch + 1 < self.n_epochs
        if self._exchange_fn is not None:
            posted = self._stager._posted
            if w not in posted or (w + 1) not in posted:
                self._ensure_posted(w)
            # the engine's cross-window lookahead reads w + 1: only once its exchange is issued
            nxt = nxt and (w + 1) in posted
        if _TRACE_ENGINE:  # roctx range per native get (DDL_ROCTX=2: host timeline under rocprofv3)
            with trace_range("ddl.engine.get"):
                slot, prod, tags = eng.get(w, local, bpw, nxt, handle, self._timeout_ms)
        else:
            slot, prod, tags = eng.get(w, local, bpw, nxt, handle, self._timeout_ms)
        if slot < 0:
            self._engine_raise(slot, prod, f"batch {local} of window {w}")
        if local == 0 and self._verify is not None:
            self._verify_window(w, tags)
        if self._eng_window != w:
            self._eng_window = w
            self._eng_given.clear()
            self._eng_spare.clear()
            self.metrics.windows += 1
        spare = self._eng_spare.pop(slot, None) if self._eng_spare else None
        if spare is not None:  # whole-window mode: a batch of this window fetched after a later one
            out, block = spare
        else:
            q = self._eng_slots
            while q[0][0] != slot:  # slots the engine skipped (dropped lookahead; whole-window: fetched later)
                sid, o, b = q.popleft()
                if self._eng_whole:
                    self._eng_spare[sid] = (o, b)
            _, out, block = q.popleft()
        self._eng_given[local] = (out, block, tags)
        if self._eng_rec[0] is not block or self._eng_rec[1] is not cur:
            block.record_stream(cur)  # the compute stream uses this block from now on
            self._eng_rec = (block, cur)
        return self._engine_outputs(out, tags)

    def _engine_outputs(self, out, tags):
        if self._eng_tokens is None:
            return (out[0],) if self._eng_aug else out
        n_tokens, n_rows, n_seg, max_seg = tags
        if self._eng_tokens == "pad":
            return {"input_ids": out[0], "attention_mask": out[1], "position_ids": out[2], "n_tokens": n_tokens}
        if n_tokens > 0x7FFFFFFF:
            raise ValueError(f"{n_tokens} tokens in one batch overflow int32 cu_seqlens")
        if self.token_rows == "fixed":
            return {"input_ids": out[0], "attention_mask": out[1], "position_ids": out[2], "segment_ids": out[3],
                    "cu_seqlens": out[4][:n_seg + 1], "max_seqlen": max_seg, "n_tokens": n_tokens, "n_rows": n_rows}
        return {"input_ids": out[0][:n_rows], "attention_mask": out[1][:n_rows], "position_ids": out[2][:n_rows],
                "segment_ids": out[3][:n_rows], "cu_seqlens": out[4][:n_seg + 1], "max_seqlen": max_seg,
                "n_tokens": n_tokens}

    def _native_stats(self, d: dict) -> None:
        """The native engine's counters into the loader's ``stats()`` dict ``d`` (``native_dispatch``)."""
        done = getattr(self, "_native_done", None)
        if self._engine is not None or done is not None:
            nd = dict(done or {"batches": 0, "lookahead_hits": 0})
            if self._engine is not None:
                d["consumer_wait_s"] += self._engine.wait_s
                nd["batches"] += int(self._engine.batches)
                nd["lookahead_hits"] += int(self._engine.lookahead_hits)
                g, la, rec, sw = self._engine.timing_ns
                n = max(1, int(self._engine.batches))
                nd["compute_waits"] = int(self._engine.compute_waits)
                nd["ready_host_waits"] = int(self._engine.ready_host_waits)
                wait_ns = self._engine.wait_s * 1e9
                nd["host_us_per_batch"] = {"get": round(g / n / 1e3, 2),
                                           "get_excl_staging_wait": round(max(0.0, g - wait_ns) / n / 1e3, 2),
                                           "kernel_launch": round(la / n / 1e3, 2),
                                           "event_record": round(rec / n / 1e3, 2),
                                           "stream_wait": round(sw / n / 1e3, 2)}
            nd["mode"] = getattr(self, "_eng_mode", None)
            if self._engine is not None:
                nd["handoff"] = "host" if self._engine.host_handoff else "device"
            d["native_dispatch"] = nd
