"""Per-batch work of the consumer on a staged window (Python dispatch path; the native engine,
``engine_dispatch.py``, runs the same recipes in C++).

A batch of window ``w`` is rows ``[local*B, (local+1)*B)`` of the window in the window's order -- the
reference's slice of the producer's window (reference ddl/mpi_dataloader.py:179-198) -- built on the device by
one fused gfx950 kernel: Feistel permutation gather + dtype cast + per-channel normalise, HWC->CHW collate,
RandomResizedCrop + flip, contiguous column split or token collate (``ops/``). Kernels run on a batch stream
one batch ahead of the consumer (``_device_batch``); the consumer's stream only waits on an event.
"""

from __future__ import annotations

import math

import torch

from . import ops
from .permutation import FeistelPermutation
from .utils import streams
from .utils.tracing import trace_range


def _mix(a: int, b: int) -> int:
    """64-bit mix of two ints (splitmix64 finaliser over a*phi + b)."""
    z = (int(a) * 0x9E3779B97F4A7C15 + int(b) + 0x632BE59BD9B4E019) & ((1 << 64) - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return z ^ (z >> 31)


def window_perm_key(producer: int, round_: int) -> int:
    """Key of the device permutation of one window visit (producer ``p``, round ``seq``): a 64-bit
    mix of both, so every (producer, round) pair has its own order at any producer count."""
    return _mix(producer, round_) & ((1 << 63) - 1)


class WindowBatchMixin:
    """Batch construction over ``self._stager`` windows (host views on the CPU path)."""

    def _unpack(self, out):
        from .models.datasets import unpack_fields

        rows = out[0] if isinstance(out, (tuple, list)) else out
        return unpack_fields(rows, *self._fields)

    # ---------------------------------------------------------- batch stream
    def _produces_copy(self) -> bool:
        """True when a batch is built by a kernel (not a zero-copy view of the window)."""
        return (self.shuffle == "device" or self.out_dtype not in (None, self.window_dtype) or self.augment is not None
                or self.normalize is not None or self.copy_batches or self.contiguous or self.collate is not None)

    def _enqueue_batch(self, sw, p: int, s: int, local: int):
        """Build batch ``local`` of window ``sw`` on the batch stream; returns (outputs, ready event)."""
        bs = self._batch_stream
        self._stager.wait_ready(sw, bs)
        with streams.on_stream(bs):
            out = self._batch_from_window(sw, p, s, local)
            ev = torch.cuda.Event()
            ev.record(bs)
        if local + 1 == self.batches_per_window[p]:
            # the window's free event: right after its last batch kernel, NOT at release time behind the
            # next window's lookahead kernel (which waits for that window's copy: the copy after it would
            # then wait for a copy plus a gather)
            self._win_done[sw.index] = ev
        return out, ev

    def _device_batch(self, sw, p: int, s: int, local: int, bpw: int):
        """Batch kernels run on their own stream one batch ahead of the consumer:
        batch l+1's gather overlaps the training step on batch l, and the compute
        stream only waits on an event (no host sync)."""
        hit = self._lookahead.pop((self.window, local), None)
        out, ev = hit if hit is not None else self._enqueue_batch(sw, p, s, local)
        cur = streams.current(self.device.index)
        cur.wait_event(ev)
        for t in (out.values() if isinstance(out, dict) else out):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(cur)
        if local + 1 < bpw:
            if (self.window, local + 1) not in self._lookahead:
                self._lookahead[(self.window, local + 1)] = self._enqueue_batch(sw, p, s, local + 1)
        elif self.window_in_epoch + 1 < self.windows_per_epoch or self.epoch + 1 < self.n_epochs:
            # last batch of this window: start the next window's first batch if it is already in HBM
            nxt = self._stager.peek(self.window + 1)
            if nxt is not None and (self.window + 1, 0) not in self._lookahead:
                np_, ns = self._schedule(self.window + 1)
                self._lookahead[(self.window + 1, 0)] = self._enqueue_batch(nxt, np_, ns, 0)
        return out

    def _perm_for(self, p: int, seq: int) -> FeistelPermutation | None:
        if self.shuffle != "device":
            return None
        # key = (seed, producer, round): every window visit gets a fresh order.
        return FeistelPermutation(self.metadata_from_producer[p].nData, self.seed, window_perm_key(p, seq))

    def _batch_from_window(self, sw, p: int, s: int, local: int):
        B = self.batch_size
        n_data = self.shapes[p][0]
        wdt = self.window_dtype
        if sw is None:  # host path: zero-copy views of the shm window
            _, win = self.arys[p][s]
            seq, tags = self._host_seq, self._host_tags
            meta = getattr(self, "_host_meta", ())
        else:
            win = sw.data.view(wdt).view((n_data,) + self.sample_shape) if self.collate is None else sw.data
            seq, tags, meta = sw.seq, sw.tags, sw.meta
        if self.collate == "tokens":
            from .models.tokens import TokenWindowLayout, collate_token_window

            ex = self.metadata_from_producer[p].extra
            with trace_range("ddl.consumer.tokens"):
                return collate_token_window(win.reshape(-1), TokenWindowLayout(**ex["token_layout"]),
                                            ex["token_mode"], meta, self.pad_id, sub=local,
                                            fixed_rows=self.token_rows == "fixed")
        perm = self._perm_for(p, seq)
        out_dtype = self.out_dtype or (torch.float32 if self.normalize is not None else wdt)
        if self.augment is not None:
            aug, norm = self.augment, self.normalize or {}
            # crop randomness keyed by (seed, epoch OF THIS WINDOW) and the row's identity (producer, round, row);
            # the window's epoch, not the cursor's: a lookahead batch of the next window is built a step early
            w = sw.index if sw is not None else self.window
            epoch = self.epoch + (w - (self.window - self.window_in_epoch)) // self.windows_per_epoch
            return (ops.random_resized_crop(
                win, perm=perm, base=local * B, n_rows=B, size=aug.get("size", (224, 224)),
                scale=aug.get("scale", (0.08, 1.0)), ratio=aug.get("ratio", (3.0 / 4.0, 4.0 / 3.0)),
                flip_p=aug.get("flip_p", 0.5), seed=_mix(self.seed, epoch),
                sample_base=_mix(p, seq) & ~0xFFFFFFFF & ((1 << 63) - 1), layout=aug.get("layout", "chw"),
                out_dtype=self.out_dtype or torch.bfloat16, mean=norm.get("mean"), std=norm.get("std")),)
        splits = list(self.splits[p])
        norm = self.normalize
        with trace_range("ddl.consumer.batch"):
            if norm is not None and norm.get("layout", "chw") == "hwc":
                x = ops.collate_hwc_to_chw(win, perm=perm, base=local * B, n_rows=B, out_dtype=out_dtype,
                                           mean=norm.get("mean"), std=norm.get("std"))
                return (x,)
            if (self.contiguous or self.copy_batches) and len(splits) > 1 and len(self.sample_shape) == 1 \
                    and norm is None:
                return ops.split_columns(win, splits, perm=perm, base=local * B, n_rows=B, out_dtype=out_dtype)
            if perm is None and out_dtype == wdt and norm is None and not self.copy_batches:
                x = win[local * B:(local + 1) * B]  # zero-copy view (reference semantics)
            else:
                kw = {}
                if norm is not None:
                    plane = int(math.prod(self.sample_shape[1:])) if len(self.sample_shape) > 1 else 1
                    c = self.sample_shape[0] if len(self.sample_shape) > 1 else len(norm.get("mean", [0]))
                    sc, bi = ops.norm_affine(c, norm.get("mean"), norm.get("std"), norm.get("scale"),
                                             norm.get("bias"), ops.pixel_max(wdt))
                    kw = dict(scale=sc, bias=bi, plane=plane)
                x = ops.gather_rows(win, perm=perm, base=local * B, n_rows=B, out_dtype=out_dtype, **kw)
        if len(splits) == 1:
            return (x,)
        parts = torch.split(x.reshape(B, -1), splits, dim=1)
        if self.contiguous or self.copy_batches:  # normalised tabular rows: own each column group
            return tuple(t.contiguous() for t in parts)
        return parts
