"""Token-sequence family (BASELINE config 4: seq_len = 4096, on-device pad/pack).

The producer ships the batch RAGGED -- flat tokens + int64 offsets (+ the
pack plan) -- so PCIe carries only real tokens (a padded [B, 4096] batch of
sequences averaging 2k tokens would double the bytes); the consumer expands it
on the GPU with the ``pad_pack_tokens`` gfx950 kernel into
``tokens [R, S]``, ``attention_mask [R, S]``, ``position_ids [R, S]`` (+
``segment_ids`` / ``cu_seqlens`` / ``max_seqlen`` in pack mode).

Pack-mode varlen metadata follows the varlen-attention ABI: ``cu_seqlens`` is
int32 ``[n_seg + 1]`` and indexes the UNPADDED token stream
``input_ids[attention_mask.bool()]`` (row-major; rows are packed in segment
order and padded only at their ends), one entry per *segment*: a sequence
longer than ``seq_len`` is split into ``seq_len`` chunks, each its own segment
with its own position ids, and empty sequences have no segment.
``max_seqlen`` is the longest segment (a Python int, from the producer).
Every batch also carries ``n_tokens``: the real tokens shipped for it.

Tokens are int32 in the corpus and on the wire, or uint16 when every id is below 65536
(``SharedTokenSource.create(..., token_dtype="auto")``: GPT-2-sized vocabularies): half the bytes per
token cross PCIe -- the token feed is link-bound, like the image feed -- and the pad/pack kernel widens
them to int32 ``input_ids`` as it writes them, so the model sees the same batch.

Sequence order is the world-size-invariant ``EpochOrder`` over sequences, so
token batches share the indexed-mode checkpoint format.
"""

from __future__ import annotations

import dataclasses
import functools

import numpy as np
import torch

from ..datapusher import DataProducerOnInitReturn
from ..datasetwrapper import ProducerFunctionSkeleton
from .. import _native
from ..permutation import EpochOrder
from .datasets import SharedArraySource


META_FIELDS = 5  # per sub-batch: n_tokens, n_rows, n_seg, max_seg, token start (elements into the tokens region)


@functools.lru_cache(maxsize=64)
def _regions(batch: int, max_segments: int, max_len: int, k: int, token_bytes: int = 4) -> dict[str, tuple[int, int]]:
    """name -> (byte offset, element count): the meta table, sub-batch 0's header arrays (sub-batch j's are
    ``header_stride`` bytes further), the shared tokens region; ``_header_stride`` and ``_total`` bytes."""
    out, off = {"meta": (0, META_FIELDS * k)}, -(-META_FIELDS * k * 8 // 16) * 16
    hdr0 = off
    for name, count in (("offsets", batch + 1), ("row_start", max_segments), ("row_end", max_segments),
                        ("seg_offsets", max_segments + 1)):
        out[name] = (off, count)
        off += count * 8
    stride = -(-(off - hdr0) // 16) * 16
    off = hdr0 + k * stride
    out["tokens"] = (off, k * batch * max_len)
    off += -(-k * batch * max_len * token_bytes // 16) * 16
    out["_header_stride"] = (stride, 0)
    out["_total"] = (off, 0)
    return out


@dataclasses.dataclass(frozen=True)
class TokenWindowLayout:
    """Byte layout of one token window: ``k`` consecutive local batches (all regions 8-byte aligned).

    ``meta`` [k, 5] int64 (n_tokens, n_rows, n_seg, max_seg, token start of each sub-batch) comes first:
    the stager copies it on the host at staging time (``meta_bytes``), so the consumer knows every
    sub-batch's sizes without reading the device copy. Then one header block per sub-batch (sequence
    offsets, packing plan), then the sub-batches' tokens back to back (only used bytes cross PCIe).
    """

    batch: int      # sequences per (local) batch
    seq_len: int    # S
    max_len: int    # longest sequence in the corpus
    k: int = 1      # batches per window
    token_bytes: int = 4  # 4: int32 tokens, 2: uint16 (widened on the device)

    @property
    def max_segments(self) -> int:
        return self.batch * max(1, -(-self.max_len // self.seq_len))

    def regions(self) -> dict[str, tuple[int, int]]:
        """name -> (byte offset, element count). Computed once per layout (per-batch host path)."""
        return _regions(self.batch, self.max_segments, self.max_len, self.k, self.token_bytes)

    @property
    def nbytes(self) -> int:
        return self.regions()["_total"][0]

    @property
    def header_stride(self) -> int:
        return self.regions()["_header_stride"][0]

    @property
    def meta_bytes(self) -> int:
        return META_FIELDS * self.k * 8

    @property
    def row_bytes(self) -> int:
        return -(-self.nbytes // (self.batch * self.k) // 16) * 16

    def views(self, buf: torch.Tensor, sub: int = 0) -> dict[str, torch.Tensor]:
        """Typed views of a uint8 window buffer (host or device): sub-batch ``sub``'s header arrays, the
        whole tokens region and the meta table [k, 5]."""
        v = {}
        stride = self.header_stride * sub
        for name, (off, count) in self.regions().items():
            if name.startswith("_"):
                continue
            if name == "tokens":
                tb = self.token_bytes
                v[name] = buf[off:off + count * tb].view(torch.int32 if tb == 4 else torch.int16)
            elif name == "meta":
                v[name] = buf[off:off + count * 8].view(torch.int64).view(self.k, META_FIELDS)
            else:
                v[name] = buf[stride + off:stride + off + count * 8].view(torch.int64)
        return v


class SharedTokenSource:
    """A tokenised corpus in node-wide shm: flat tokens (int32, or uint16 ids stored as int16) + int64
    sequence offsets."""

    def __init__(self, tokens: SharedArraySource, offsets: SharedArraySource, max_len: int):
        self.tokens, self.offsets, self.max_len = tokens, offsets, int(max_len)
        self.n = offsets.n - 1
        self.token_bytes = 2 if tokens.dtype in (torch.int16, torch.uint16) else 4

    @classmethod
    def create(cls, name: str, tokens: np.ndarray, offsets: np.ndarray,
               token_dtype: str = "int32") -> "SharedTokenSource":
        """``token_dtype``: "int32", "uint16" (every id must be < 65536) or "auto" (uint16 when they are)."""
        tokens = np.asarray(tokens)
        if token_dtype not in ("int32", "uint16", "auto"):
            raise ValueError("token_dtype must be 'int32', 'uint16' or 'auto'")
        fits = tokens.size == 0 or (int(tokens.min()) >= 0 and int(tokens.max()) < 65536)
        if token_dtype == "uint16" and not fits:
            raise ValueError("token ids outside [0, 65536) cannot be stored as uint16")
        if token_dtype == "uint16" or (token_dtype == "auto" and fits):
            tok = torch.from_numpy(np.ascontiguousarray(tokens, np.uint16).view(np.int16)).view(-1, 1)
        else:
            tok = torch.from_numpy(np.ascontiguousarray(tokens, np.int32)).view(-1, 1)
        off = torch.from_numpy(np.ascontiguousarray(offsets, np.int64)).view(-1, 1)
        t = SharedArraySource.create(name + "_tok", tok)
        o = SharedArraySource.create(name + "_off", off)
        return cls(t, o, int(np.diff(offsets).max()) if len(offsets) > 1 else 0)

    @classmethod
    def synthetic(cls, name: str, n: int, min_len: int = 128, max_len: int = 4096, vocab: int = 50257,
                  seed: int = 0, token_dtype: str = "int32") -> "SharedTokenSource":
        rng = np.random.default_rng(seed)
        lens = rng.integers(min_len, max_len + 1, size=n).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        toks = rng.integers(0, vocab, size=int(offs[-1]), dtype=np.int32)
        return cls.create(name, toks, offs, token_dtype)

    def bind_to_node(self, node: int | None) -> int:
        """Place the corpus on NUMA ``node`` (pages migrate; see ``SharedArraySource.bind_to_node``): the
        producers' ragged gathers are latency-bound reads of ~8 KB runs, which cost far more from the
        other socket. ``None`` (node unknown) is a no-op. 0 or -errno."""
        if node is None:
            return 0
        return self.tokens.bind_to_node(node) or self.offsets.bind_to_node(node)

    def close(self) -> None:
        self.tokens.close()
        self.offsets.close()


def ffd_order(lengths: np.ndarray, seq_len: int) -> tuple[np.ndarray, int]:
    """First-fit-decreasing order of one batch's sequences (native ``ffd_order`` in
    ``csrc/runtime/arena.cpp``; ``ffd_order_py`` is its NumPy reference)."""
    order, n_rows = _native.runtime().ffd_order(np.ascontiguousarray(lengths, dtype=np.int64), int(seq_len))
    return order, int(n_rows)


def in_order_rows(lengths: np.ndarray, seq_len: int) -> int:
    """Rows that in-order packing (``pack_plan``) of sequences of these lengths produces:
    over-long sequences become ``seq_len`` chunks, a row breaks where the next segment does not fit.
    Native (``_ddl_runtime.in_order_rows``); ``in_order_rows_py`` is its reference."""
    return int(_native.runtime().in_order_rows(np.ascontiguousarray(lengths, dtype=np.int64), int(seq_len)))


def in_order_rows_py(lengths: np.ndarray, seq_len: int) -> int:
    S = int(seq_len)
    rows, cur = 0, S  # cur = tokens in the open row (S: no open row)
    for n in np.asarray(lengths, dtype=np.int64).tolist():
        while n > 0:
            seg = min(n, S)
            if cur + seg > S:
                rows += 1
                cur = 0
            cur += seg
            n -= seg
    return rows


def ffd_order_py(lengths: np.ndarray, seq_len: int) -> tuple[np.ndarray, int]:
    """First-fit-decreasing bin packing of sequences into rows of ``seq_len`` tokens.

    Returns the batch-local sequence order and the number of rows that in-order
    packing (``pack_plan``) of that order produces. A sequence longer than ``seq_len``
    takes ``L // seq_len`` full rows; its remainder ``L % seq_len`` is packed like a
    short sequence, into a bin that holds no other remainder, and the whole sequence
    is emitted at the head of that bin, so its tokens stay contiguous. Each other bin
    lists its sequences longest first. In-order packing of the result therefore
    breaks rows exactly at bin boundaries. A bin's first item is either a full chunk,
    which fits nowhere, or the bin's longest sequence, which did not fit in any earlier
    bin when it was placed (earlier bins only fill up).
    """
    lengths = np.asarray(lengths, dtype=np.int64)
    S = int(seq_len)
    rem_len = np.where(lengths > S, lengths % S, lengths)
    full = np.where(lengths > S, lengths // S, 0)
    items = np.nonzero(rem_len > 0)[0]
    items = items[np.argsort(-rem_len[items], kind="stable")]
    left = np.empty(len(items), dtype=np.int64)
    has_long = np.zeros(len(items), dtype=bool)
    bins: list[list[int]] = []
    for i in items:
        is_long = lengths[i] > S
        ok = left[: len(bins)] >= rem_len[i]
        if is_long:
            ok &= ~has_long[: len(bins)]
        fit = np.nonzero(ok)[0]
        if len(fit):
            b = int(fit[0])
        else:
            b = len(bins)
            bins.append([])
            left[b] = S
            has_long[b] = False
        bins[b].append(int(i))
        left[b] -= rem_len[i]
        has_long[b] |= is_long
    order: list[int] = []
    for members in bins:
        head = [i for i in members if lengths[i] > S]  # at most one: its full chunks, then its remainder
        order += head + [i for i in members if lengths[i] <= S]
    exact = [int(i) for i in np.nonzero(rem_len == 0)[0]]  # only full chunks, or empty
    order += exact
    return np.asarray(order, dtype=np.int64), len(bins) + int(full.sum())


class TokenBatchProducer(ProducerFunctionSkeleton):
    """One window = this rank's slice of a global batch of sequences, shipped ragged.

    ``pack_order="ffd"`` (pack mode) reorders the batch's sequences by first-fit
    decreasing before the ragged gather, so rows are packed bins: density rises
    from ~75% (in-order packing of lengths uniform in [128, 4096]) to ~93%; the order is computed natively
    (``ffd_order`` in ``csrc/runtime/arena.cpp``).
    The batch holds the same sequences, and the cursor and checkpoint are unchanged.
    """

    def __init__(self, source: SharedTokenSource, global_batch: int, seq_len: int = 4096, mode: str = "pad",
                 seed: int | None = None, host_threads: int = 2, pack_order: str = "in_order",
                 batches_per_window: int = 1):
        super().__init__()
        if batches_per_window < 1:
            raise ValueError("batches_per_window must be >= 1")
        self.batches_per_window = int(batches_per_window)
        if mode not in ("pad", "pack"):
            raise ValueError("mode must be 'pad' or 'pack'")
        if pack_order not in ("in_order", "ffd"):
            raise ValueError("pack_order must be 'in_order' or 'ffd'")
        if pack_order != "in_order" and mode != "pack":
            raise ValueError(f"pack_order={pack_order!r} reorders rows of a PACKED batch; mode={mode!r} has "
                             "one sequence per row")
        self.pack_order = pack_order
        self.source, self.global_batch, self.seq_len, self.mode, self.seed = source, global_batch, seq_len, mode, seed
        self.host_threads = host_threads
        self.order = None
        self.layout = None
        self._views: dict = {}

    def on_init(self, *args, **kwargs):
        super().on_init(*args, **kwargs)
        self.world_size = int(kwargs.get("world_size", 1))
        if self.seed is None:
            self.seed = int(kwargs.get("seed", 0))
        self.order = EpochOrder(self.source.n, self.global_batch, int(self.seed))
        lb = self.order.local_batch(self.world_size)
        bpe = self.order.batches_per_epoch
        # k consecutive global batches per window (per-window costs -- producer round, H2D, stager and
        # window hand-off -- amortised over k batches); k divides the epoch so windows never straddle it
        k = max(d for d in range(1, min(self.batches_per_window, bpe) + 1) if bpe % d == 0)
        self.layout = TokenWindowLayout(lb, self.seq_len, self.source.max_len, k, self.source.token_bytes)
        rb = self.layout.row_bytes
        return DataProducerOnInitReturn(k * lb, rb, (k * lb, rb), (rb,), "uint8", extra={
            "batches_per_epoch": bpe, "windows_per_epoch": bpe // k, "batches_per_window": k,
            "global_batch": self.global_batch, "n_samples": self.source.n, "order_seed": int(self.seed),
            "token_layout": dataclasses.asdict(self.layout), "token_mode": self.mode,
            "meta_bytes": self.layout.meta_bytes})

    def _window_views(self, buf: torch.Tensor):
        """Per staging buffer (cached): raw addresses of every sub-batch's header arrays and of the tokens
        region, and numpy views of the meta table and of the seg_offsets arrays (the producer loop below
        makes no tensor op per batch)."""
        key = (buf.data_ptr(), buf.numel())
        hit = self._views.get(key)
        if hit is None:
            lay = self.layout
            subs = []
            for j in range(lay.k):
                v = lay.views(buf, j)
                subs.append((v["offsets"].data_ptr(), v["row_start"].data_ptr(), v["row_end"].data_ptr(),
                             v["seg_offsets"].data_ptr(), v["seg_offsets"].numpy()))
            v0 = lay.views(buf, 0)
            hit = (subs, v0["meta"].numpy(), v0["tokens"].data_ptr(), v0["tokens"].numel(), buf)
            if len(self._views) >= 8:  # a producer cycles through its n_slots buffers
                self._views.clear()
            self._views[key] = hit
        return hit

    def execute_function(self, *args, **kwargs):
        rnd = int(kwargs.get("round", 0))
        lay, k = self.layout, self.layout.k
        subs, meta, tok_ptr, tok_cap, _ = self._window_views(kwargs["my_tensor"].view(-1))
        toks = self.source.tokens.tensor().view(-1)
        offs = self.source.offsets.tensor().view(-1)
        offs_all = offs.numpy()
        toks_ptr, offs_ptr, n_src = toks.data_ptr(), offs.data_ptr(), self.source.n
        rt = _native.runtime()
        base = (rnd * (self.n_producers or 1) + (self.producer_index or 0)) * k
        rank, world, bpe, S = self.rank_global or 0, self.world_size, self.order.batches_per_epoch, self.seq_len
        tb = lay.token_bytes
        pack, ffd, cap = self.mode == "pack", self.pack_order == "ffd", lay.max_segments
        tok0 = 0
        for j in range(k):
            epoch, g = divmod(base + j, bpe)
            idx = np.asarray(self.order.indices(epoch, g, rank, world), dtype=np.int64)
            if pack and ffd:
                lens = offs_all[idx + 1] - offs_all[idx]
                order, ffd_rows = ffd_order(lens, S)
                if ffd_rows < in_order_rows(lens, S):  # FFD is a heuristic: keep it only if it wins
                    idx = idx[order]
            o_ptr, rs_ptr, re_ptr, so_ptr, so_np = subs[j]
            # native ragged gather (thread pool, GIL released): sequences -> window, offsets alongside
            n_tokens = int(rt.gather_ragged(tok_ptr + tb * tok0, o_ptr, toks_ptr, offs_ptr, n_src,
                                            np.ascontiguousarray(idx, np.int64), tb, tok_cap - tok0,
                                            self.host_threads))
            n_rows = n_seg = max_seg = 0
            if pack:  # packing plan written straight into the window (native)
                n_rows, n_seg = rt.pack_plan(o_ptr, len(idx), S, rs_ptr, re_ptr, cap, so_ptr, cap)
                if n_seg:
                    max_seg = int(np.diff(so_np[: n_seg + 1]).max())
            meta[j] = (n_tokens, n_rows, n_seg, max_seg, tok0)
            tok0 += n_tokens
        tok_off = lay.regions()["tokens"][0]
        return {"tags": [tok0, k, 0, 0], "used_bytes": tok_off + tb * tok0}


_VIEW_CACHE: dict = {}


def _cached_views(buf: torch.Tensor, layout: TokenWindowLayout, sub: int = 0) -> dict[str, torch.Tensor]:
    """``layout.views(buf, sub)`` memoised per (buffer address, size, layout, sub-batch): the consumer
    collates out of the same few staging buffers every step, and building the views costs ~9 us per
    batch. A cached view keeps its (window-sized) buffer alive, so no other allocation can take that
    address while the entry exists; the cache is bounded."""
    key = (buf.data_ptr(), buf.numel(), buf.device, layout, sub)
    v = _VIEW_CACHE.get(key)
    if v is None:
        if len(_VIEW_CACHE) >= 256:
            _VIEW_CACHE.clear()
        v = _VIEW_CACHE[key] = layout.views(buf, sub)
    return v


def drop_cached_views(base_ptrs) -> int:
    """Forget the cached views of buffers starting at ``base_ptrs`` (a staging ring being dropped: a
    live seek or close), so the cache does not keep the old ring's HBM alive. Returns entries dropped."""
    ptrs = set(int(p) for p in base_ptrs)
    dead = [k for k in _VIEW_CACHE if k[0] in ptrs]
    for k in dead:
        del _VIEW_CACHE[k]
    return len(dead)


def collate_token_window(buf: torch.Tensor, layout: TokenWindowLayout, mode: str, meta, pad_id: int = 0,
                         sub: int = 0, fixed_rows: bool = False):
    """Expand sub-batch ``sub`` of one (device or host) token window into model inputs; ``meta`` is the
    window's meta table (flat, META_FIELDS per sub-batch: the stager's host copy, or the host window).
    ``fixed_rows`` (pack mode): every batch has ``layout.max_segments`` rows, the rows past the packed
    ones are padding (static shapes), and ``n_rows`` gives the packed count."""
    from .. import ops

    v = _cached_views(buf.view(-1), layout, sub)
    n_tokens, n_rows, n_seg, max_seqlen, tok0 = (int(x) for x in meta[META_FIELDS * sub:META_FIELDS * (sub + 1)])
    tokens = v["tokens"][tok0:tok0 + n_tokens]
    if mode == "pad":
        ids, mask, pos = ops.pad_tokens(tokens, v["offsets"], layout.seq_len, pad_id)
        # n_tokens: tokens shipped (pad mode truncates sequences longer than seq_len: mask.sum() can be less)
        return {"input_ids": ids, "attention_mask": mask, "position_ids": pos, "n_tokens": n_tokens}
    fill = layout.max_segments if fixed_rows else 0
    extra = {"n_rows": n_rows} if fixed_rows else {}
    if not tokens.is_cuda:
        ids, mask, pos, seg = ops.ref_pack_tokens(tokens, v["row_start"][:n_rows].numpy(),
                                                  v["row_end"][:n_rows].numpy(), v["seg_offsets"][: n_seg + 1].numpy(),
                                                  layout.seq_len, pad_id, fill_rows=fill)
        return {"input_ids": ids, "attention_mask": mask, "position_ids": pos, "segment_ids": seg,
                "cu_seqlens": v["seg_offsets"][: n_seg + 1].to(torch.int32), "max_seqlen": max_seqlen,
                "n_tokens": n_tokens, **extra}
    dev = tokens.device
    s = layout.seq_len
    # one allocation for all five outputs (aligned regions: position_ids i64, cu_seqlens i32,
    # input_ids i32, segment_ids i32, attention_mask u8). cu_seqlens is written by the kernel into
    # memory of its own: a view of the staging buffer would be overwritten when it is re-staged
    R = max(n_rows, fill)
    n = R * s
    cu_n = -(-(n_seg + 1) // 4) * 4  # i32 count rounded so the following regions stay 16-byte aligned
    whole = torch.empty(8 * n + 4 * cu_n + 4 * n + 4 * n + n, dtype=torch.uint8, device=dev)
    o = 0
    pos = whole[o:o + 8 * n].view(torch.int64).view(R, s)
    o += 8 * n
    cu = whole[o:o + 4 * (n_seg + 1)].view(torch.int32)
    o += 4 * cu_n
    ids = whole[o:o + 4 * n].view(torch.int32).view(R, s)
    o += 4 * n
    seg = whole[o:o + 4 * n].view(torch.int32).view(R, s)
    o += 4 * n
    mask = whole[o:o + n].view(R, s)
    from ..ops.kernels import _stream_handle

    if n_tokens > 0x7FFFFFFF:
        raise ValueError(f"{n_tokens} tokens in one batch overflow int32 cu_seqlens")
    if R == 0:
        cu.copy_(v["seg_offsets"][: n_seg + 1])
    else:
        _native.hip().pad_pack_tokens(
            tokens=tokens.data_ptr(), offsets=0, row_start=v["row_start"].data_ptr(),
            row_end=v["row_end"].data_ptr(), seg_offsets=v["seg_offsets"].data_ptr(), n_seg=n_seg,
            out_tokens=ids.data_ptr(), attn_mask=mask.data_ptr(), position_ids=pos.data_ptr(), pos_is_i64=True,
            segment_ids=seg.data_ptr(), cu_seqlens_out=cu.data_ptr(), rows=n_rows, seq_len=s, pad_id=pad_id, mode=1,
            stream=_stream_handle(None), fill_rows=fill, tok16=layout.token_bytes == 2)
    return {"input_ids": ids, "attention_mask": mask, "position_ids": pos, "segment_ids": seg, "cu_seqlens": cu,
            "max_seqlen": max_seqlen, "n_tokens": n_tokens, **extra}


def expected_tokens(source: SharedTokenSource, idx) -> list[np.ndarray]:
    toks = source.tokens.tensor().view(-1).numpy()
    if source.token_bytes == 2:  # uint16 ids stored as int16
        toks = toks.view(np.uint16).astype(np.int32)
    offs = source.offsets.tensor().view(-1).numpy()
    return [toks[offs[i]:offs[i + 1]] for i in idx]

