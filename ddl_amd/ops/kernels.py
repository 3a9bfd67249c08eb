"""Python front-end of the hand-written gfx950 kernels (csrc/kernels/*.hip).

Every op dispatches to the HIP kernel when its tensors live on the GPU and to
a plain-PyTorch reference (``ref_*``) when they live on the CPU. There is no
silent fallback on GPU: if the extension is missing on a GPU host the call
raises ``NativeExtensionError`` (see ``ddl_amd._native``). Tests compare each
kernel against its ``ref_*`` (an fp32 PyTorch reference of the same op).

Row-indexing convention shared by the gather-style ops (``RowIndex`` in
csrc/kernels/common.h): output row ``r`` reads source row
  * ``index[r]``                      if ``index`` is given,
  * ``perm(base + r)``                if ``perm`` (a FeistelPermutation) is given,
  * ``base + r``                      otherwise.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Sequence

import numpy as np
import torch

from .. import _native
from ..permutation import FeistelPermutation
from . import _dtypes


@dataclasses.dataclass
class HostRows:
    """Rows living in pinned, device-mapped host memory (zero-copy source).

    ``cpu`` is a CPU tensor view of the memory ([N, *row_shape]); ``device_ptr``
    is the address the GPU uses for it (``hipHostGetDevicePointer``).
    """

    cpu: torch.Tensor
    device_ptr: int

    @property
    def shape(self):
        return self.cpu.shape

    @property
    def dtype(self):
        return self.cpu.dtype

    @property
    def device(self):
        return torch.device("cuda", torch.cuda.current_device())

    def dim(self) -> int:
        return self.cpu.dim()


def _stream_handle(stream) -> int:
    if stream is None:
        # == torch.cuda.current_stream().cuda_stream, without building a Stream object (per-launch host cost)
        return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _is_gpu(t) -> bool:
    return isinstance(t, HostRows) or (isinstance(t, torch.Tensor) and t.is_cuda)


def _src_addr(src) -> int:
    return src.device_ptr if isinstance(src, HostRows) else src.data_ptr()


def _index_kw(index: torch.Tensor | None, perm: FeistelPermutation | None, base: int) -> dict:
    if index is not None and perm is not None:
        raise ValueError("give either index or perm, not both")
    if index is not None:
        if index.dtype != torch.int64:
            raise TypeError("index must be int64")
        if not index.is_cuda:
            raise ValueError("index must live on the GPU for a GPU gather")
        return dict(mode=1, idx=index.data_ptr(), base=0, keys=[0] * 6, n_domain=1, half_bits=1)
    if perm is not None:
        return dict(mode=2, idx=0, base=int(base), **perm.device_args())
    return dict(mode=0, idx=0, base=int(base), keys=[0] * 6, n_domain=1, half_bits=1)


def _ref_rows(n_src: int, n_rows: int, index, perm, base) -> torch.Tensor:
    if index is not None:
        return index.to("cpu", torch.int64)
    pos = np.arange(base, base + n_rows, dtype=np.int64)
    if perm is not None:
        return torch.from_numpy(perm(pos))
    if pos.size and pos.max() >= n_src:
        raise IndexError("identity rows out of range")
    return torch.from_numpy(pos)


def _affine_lists(scale, bias) -> tuple[list[float], list[float]]:
    if scale is None and bias is None:
        return [], []
    if scale is None:
        scale = [1.0] * len(bias)
    if bias is None:
        bias = [0.0] * len(scale)
    scale, bias = [float(s) for s in scale], [float(b) for b in bias]
    if len(scale) != len(bias) or not 1 <= len(scale) <= 16:
        raise ValueError("scale/bias: 1..16 channels of equal length")
    return scale, bias


def _check_rows(src, index, perm, base, n_rows) -> int:
    n_src = src.shape[0]
    if n_rows is None:
        if index is not None:
            n_rows = index.numel()
        elif perm is not None:
            n_rows = perm.n - base
        else:
            n_rows = n_src - base
    if n_rows < 0:
        raise ValueError("negative row count")
    if perm is not None and (base < 0 or base + n_rows > perm.n):
        raise IndexError("perm positions out of range")
    if perm is not None and perm.n > n_src:
        raise IndexError("permutation domain larger than the source")
    if index is None and perm is None and base + n_rows > n_src:
        raise IndexError("identity rows out of range")
    return int(n_rows)


# --------------------------------------------------------------------- gather
def ref_gather_rows(src, index=None, perm=None, base=0, n_rows=None, out_dtype=None, scale=None, bias=None,
                    plane=None) -> torch.Tensor:
    x = src.cpu if isinstance(src, HostRows) else src
    n_rows = _check_rows(x, index, perm, base, n_rows)
    rows = x.index_select(0, _ref_rows(x.shape[0], n_rows, index, perm, base).to(x.device))
    out_dtype = out_dtype or x.dtype
    sc, bi = _affine_lists(scale, bias)
    if sc:
        flat = rows.reshape(n_rows, -1).double()
        ch = (torch.arange(flat.shape[1], device=flat.device) // int(plane)) % len(sc)
        s = torch.tensor(sc, dtype=torch.float64, device=flat.device)[ch]
        b = torch.tensor(bi, dtype=torch.float64, device=flat.device)[ch]
        rows = (flat * s + b).float().reshape(rows.shape)
    elif out_dtype != x.dtype:
        rows = rows.float()
    return rows.to(out_dtype)


def gather_rows(src, index: torch.Tensor | None = None, *, perm: FeistelPermutation | None = None, base: int = 0,
                n_rows: int | None = None, out: torch.Tensor | None = None, out_dtype=None, scale=None, bias=None,
                plane: int | None = None, stream=None, max_blocks: int = 0) -> torch.Tensor:
    """out[r] = cast(affine(src[row(r)])): fused permute + cast + per-channel normalise.

    ``max_blocks`` > 0 caps the grid (the kernel grid-strides over row tiles):
    a zero-copy gather out of pinned host memory is PCIe-latency-bound and
    saturates the link with a few dozen workgroups, leaving the other CUs to
    the training step.
    """
    if out_dtype is not None:
        out_dtype = _dtypes.to_torch_dtype(out_dtype)
    else:
        out_dtype = out.dtype if out is not None else src.dtype
    if not _is_gpu(src):
        res = ref_gather_rows(src, index, perm, base, n_rows, out_dtype, scale, bias, plane)
        if out is not None:
            out.copy_(res)
            return out
        return res
    n_rows = _check_rows(src, index, perm, base, n_rows)
    row_shape = tuple(src.shape[1:])
    row_elems = int(math.prod(row_shape)) if row_shape else 1
    if isinstance(src, torch.Tensor) and not src.is_contiguous():
        raise ValueError("gather_rows: source must be contiguous")
    if out is None:
        out = torch.empty((n_rows,) + row_shape, dtype=out_dtype, device=src.device)
    elif not out.is_contiguous() or out.dtype != out_dtype or out.numel() != n_rows * row_elems:
        raise ValueError("gather_rows: bad out tensor")
    sc, bi = _affine_lists(scale, bias)
    if sc and plane is None:
        raise ValueError("plane (elements per channel) is required with scale/bias")
    if sc and (out_dtype in (torch.uint8, torch.int32, torch.int64)):
        raise TypeError("normalisation needs a floating output dtype")
    if out_dtype != src.dtype and out_dtype not in (torch.bfloat16, torch.float16, torch.float32):
        raise TypeError(f"cannot cast {src.dtype} -> {out_dtype} in the gather")
    _native.hip().gather_rows(
        dst=out.data_ptr(), out_dt=_dtypes.code(out_dtype), src=_src_addr(src), in_dt=_dtypes.code(src.dtype),
        n_rows=n_rows, row_elems=row_elems, scale=sc, bias=bi, plane=int(plane or 0), scatter=False,
        stream=_stream_handle(stream), max_blocks=int(max_blocks), host_src=isinstance(src, HostRows),
        **_index_kw(index, perm, base))
    return out


def scatter_rows(dst: torch.Tensor, src: torch.Tensor, index: torch.Tensor, *, stream=None,
                 max_blocks: int = 0) -> torch.Tensor:
    """dst[index[r]] = src[r] (same dtype). Used to put exchanged rows back. ``max_blocks`` > 0 caps the
    grid, as for ``gather_rows``."""
    if dst.dtype != src.dtype or dst.shape[1:] != src.shape[1:]:
        raise ValueError("scatter_rows: dst/src row mismatch")
    if index.numel() != src.shape[0]:
        raise ValueError("scatter_rows: one index per source row")
    if not dst.is_cuda:
        dst.index_copy_(0, index.to(torch.int64), src)
        return dst
    row_elems = int(math.prod(src.shape[1:])) if src.dim() > 1 else 1
    _native.hip().gather_rows(
        dst=dst.data_ptr(), out_dt=_dtypes.code(dst.dtype), src=src.data_ptr(), in_dt=_dtypes.code(src.dtype),
        n_rows=src.shape[0], row_elems=row_elems, scale=[], bias=[], plane=0, scatter=True,
        stream=_stream_handle(stream), max_blocks=int(max_blocks), **_index_kw(index, None, 0))
    return dst


def feistel_indices(perm: FeistelPermutation, base: int, count: int, device=None, stream=None) -> torch.Tensor:
    """Materialise perm(base .. base+count-1) (int64) on ``device``."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    if base < 0 or base + count > perm.n:
        raise IndexError("positions out of range")
    if device.type != "cuda":
        return torch.from_numpy(perm(np.arange(base, base + count, dtype=np.int64)))
    out = torch.empty(count, dtype=torch.int64, device=device)
    _native.hip().feistel_indices(out=out.data_ptr(), count=count, base=base, stream=_stream_handle(stream),
                                  **perm.device_args())
    return out


def cast(x: torch.Tensor, dtype, *, scale=None, bias=None, plane=None, stream=None) -> torch.Tensor:
    """Vectorised dtype cast (RNE to bf16) with optional per-channel affine."""
    dtype = _dtypes.to_torch_dtype(dtype)
    rows = x.reshape(x.shape[0], -1) if x.dim() > 1 else x.reshape(1, -1)
    out = gather_rows(rows, out_dtype=dtype, scale=scale, bias=bias, plane=plane, stream=stream)
    return out.reshape(x.shape)


# -------------------------------------------------------------------- collate
def ref_collate_hwc_to_chw(src, index=None, perm=None, base=0, n_rows=None, out_dtype=torch.bfloat16, mean=None,
                           std=None, scale=None, bias=None) -> torch.Tensor:
    x = src.cpu if isinstance(src, HostRows) else src
    n_rows = _check_rows(x, index, perm, base, n_rows)
    rows = x.index_select(0, _ref_rows(x.shape[0], n_rows, index, perm, base).to(x.device))
    c = rows.shape[-1]
    sc, bi = norm_affine(c, mean, std, scale, bias, pixel_max(x.dtype))
    y = rows.double().movedim(-1, 1)  # [B, C, H, W]
    if sc:
        s = torch.tensor(sc, dtype=torch.float64, device=y.device).view(1, c, *([1] * (y.dim() - 2)))
        b = torch.tensor(bi, dtype=torch.float64, device=y.device).view(1, c, *([1] * (y.dim() - 2)))
        y = y * s + b
    return y.float().to(out_dtype).contiguous()


def pixel_max(dtype) -> float:
    """Value range the mean/std convention refers to: uint8 pixels are read as x/255
    (torchvision convention on [0, 1] images); every other dtype as raw values."""
    return 255.0 if _dtypes.to_torch_dtype(dtype) == torch.uint8 else 1.0


def norm_affine(c, mean=None, std=None, scale=None, bias=None, in_max: float = 255.0):
    """(x/in_max - mean)/std  ==  x*scale + bias  with scale=1/(in_max*std), bias=-mean/std.

    ``in_max`` is ``pixel_max(source dtype)``: 255 for uint8 sources, 1 otherwise.
    """
    if mean is not None or std is not None:
        mean = list(mean) if mean is not None else [0.0] * c
        std = list(std) if std is not None else [1.0] * c
        if len(mean) != c or len(std) != c:
            raise ValueError("mean/std must have one entry per channel")
        return [1.0 / (in_max * s) for s in std], [-m / s for m, s in zip(mean, std)]
    return _affine_lists(scale, bias)


def collate_hwc_to_chw(src, index: torch.Tensor | None = None, *, perm: FeistelPermutation | None = None,
                       base: int = 0, n_rows: int | None = None, out_dtype=torch.bfloat16, mean=None, std=None,
                       scale=None, bias=None, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """[N, H, W, C] (u8/f32/bf16, HWC) rows -> [B, C, H, W] normalised bf16/f32 (LDS-staged de-interleave).

    ``mean``/``std`` follow the torchvision convention on [0, 1] pixels for uint8
    sources (``(x/255 - mean)/std``) and apply to raw values for float sources;
    alternatively pass a raw ``scale``/``bias``.
    """
    out_dtype = _dtypes.to_torch_dtype(out_dtype)
    if src.dim() < 3:
        raise ValueError("collate_hwc_to_chw expects [N, ..., C]")
    c = src.shape[-1]
    if not _is_gpu(src):
        res = ref_collate_hwc_to_chw(src, index, perm, base, n_rows, out_dtype, mean, std, scale, bias)
        if out is not None:
            out.copy_(res)
            return out
        return res
    n_rows = _check_rows(src, index, perm, base, n_rows)
    spatial = tuple(src.shape[1:-1])
    pixels = int(math.prod(spatial))
    sc, bi = norm_affine(c, mean, std, scale, bias, pixel_max(src.dtype))
    if out is None:
        out = torch.empty((n_rows, c) + spatial, dtype=out_dtype, device=src.device)
    _native.hip().collate_hwc_to_chw(
        dst=out.data_ptr(), out_dt=_dtypes.code(out_dtype), src=_src_addr(src), in_dt=_dtypes.code(src.dtype),
        batch=n_rows, pixels=pixels, channels=c, scale=sc, bias=bi, stream=_stream_handle(stream),
        **_index_kw(index, perm, base))
    return out


# ---------------------------------------------------------------- augment
def ref_random_resized_crop(src, boxes, size, layout: str = "chw", index=None, perm=None, base=0, n_rows=None,
                            out_dtype=torch.bfloat16, mean=None, std=None) -> torch.Tensor:
    """Torch reference of ``random_resized_crop`` for given crop boxes [B, 5] (y, x, h, w, flip)."""
    import torch.nn.functional as F

    x = src.cpu if isinstance(src, HostRows) else src
    n_rows = _check_rows(x, index, perm, base, n_rows)
    rows = x.index_select(0, _ref_rows(x.shape[0], n_rows, index, perm, base).to(x.device)).cpu()
    if layout == "hwc":
        rows = rows.movedim(-1, 1)
    imgs = rows.float()
    c = imgs.shape[1]
    sc, bi = norm_affine(c, mean, std, None, None, pixel_max(x.dtype))
    oh, ow = size
    out = torch.empty((n_rows, c, oh, ow), dtype=torch.float32)
    for i, (y0, x0, h, w, flip) in enumerate(boxes.tolist()):
        crop = imgs[i:i + 1, :, y0:y0 + h, x0:x0 + w]
        r = F.interpolate(crop, size=(oh, ow), mode="bilinear", align_corners=False, antialias=False)[0]
        if flip:
            r = r.flip(-1)
        if sc:
            r = r * torch.tensor(sc).view(c, 1, 1) + torch.tensor(bi).view(c, 1, 1)
        out[i] = r
    return out.to(out_dtype)


def random_resized_crop(src, index: torch.Tensor | None = None, *, perm: FeistelPermutation | None = None,
                        base: int = 0, n_rows: int | None = None, size=(224, 224), scale=(0.08, 1.0),
                        ratio=(3.0 / 4.0, 4.0 / 3.0), flip_p: float = 0.5, seed: int = 0, sample_base: int = 0,
                        layout: str = "chw", out_dtype=torch.bfloat16, mean=None, std=None,
                        return_boxes: bool = False, impl: str = "auto", stream=None,
                        sample_ids: torch.Tensor | None = None):
    """Gathered images -> RandomResizedCrop + horizontal flip + normalise + cast, one gfx950 kernel.

    ``src`` rows are [C, H, W] (``layout="chw"``) or [H, W, C] (``"hwc"``),
    uint8 / bf16 / f32. Crop boxes follow torchvision's RandomResizedCrop
    (``scale``, ``ratio``) and are drawn on the device from
    hash(``seed``, ``sample_base`` + source row): the same sample gets the same
    crop under the same seed whichever rank or batch it lands in.
    Returns [B, C, size[0], size[1]] (and the [B, 5] int32 boxes y, x, h, w,
    flip with ``return_boxes``). ``impl``: ``"auto"`` stages each band of
    output rows' source pixels in LDS when the band fits the kernel's LDS
    budget, ``"lds"`` requires that (ValueError otherwise), ``"direct"`` reads
    every tap from global memory; all three give identical results.
    ``sample_ids`` (int64 [B] on the device) replaces the source row in the crop
    key: rows gathered out of an exchange buffer keep the crop of their global
    sample id.
    """
    paths = {"auto": 0, "lds": 1, "direct": 2}
    if impl not in paths:
        raise ValueError(f"impl must be one of {sorted(paths)}")
    out_dtype = _dtypes.to_torch_dtype(out_dtype)
    if layout not in ("chw", "hwc") or src.dim() != 4:
        raise ValueError("random_resized_crop expects [N, C, H, W] (chw) or [N, H, W, C] (hwc) rows")
    if not _is_gpu(src):
        raise RuntimeError("random_resized_crop runs on the GPU (crop boxes are drawn on the device)")
    if out_dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("random_resized_crop writes bf16 or f32")
    n_rows = _check_rows(src, index, perm, base, n_rows)
    if layout == "hwc":
        h, w, c = src.shape[1:]
    else:
        c, h, w = src.shape[1:]
    oh, ow = (int(size), int(size)) if isinstance(size, int) else (int(size[0]), int(size[1]))
    sc, bi = norm_affine(c, mean, std, None, None, pixel_max(src.dtype))
    dev = src.device if isinstance(src, torch.Tensor) else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((n_rows, c, oh, ow), dtype=out_dtype, device=dev)
    boxes = torch.empty((n_rows, 5), dtype=torch.int32, device=dev)  # drawn by a per-image pre-pass
    ids_ptr = 0
    if sample_ids is not None:
        if sample_ids.dtype != torch.int64 or sample_ids.device != dev or sample_ids.numel() != n_rows \
                or not sample_ids.is_contiguous():
            raise ValueError("sample_ids must be a contiguous int64 [n_rows] tensor on the source's device")
        ids_ptr = sample_ids.data_ptr()
    _native.hip().random_resized_crop(
        dst=out.data_ptr(), out_dt=_dtypes.code(out_dtype), src=_src_addr(src), in_dt=_dtypes.code(src.dtype),
        batch=n_rows, hwc=layout == "hwc", in_h=int(h), in_w=int(w), channels=int(c), out_h=oh, out_w=ow,
        seed=int(seed) & ((1 << 64) - 1), sample_base=int(sample_base), scale_min=float(scale[0]),
        scale_max=float(scale[1]), ratio_min=float(ratio[0]), ratio_max=float(ratio[1]), flip_p=float(flip_p),
        scale=sc, bias=bi, boxes_out=boxes.data_ptr(), path=paths[impl], stream=_stream_handle(stream),
        sample_ids=ids_ptr, **_index_kw(index, perm, base))
    return (out, boxes) if return_boxes else out


def ref_split_columns(src, splits, index=None, perm=None, base=0, n_rows=None, out_dtype=None):
    x = src.cpu if isinstance(src, HostRows) else src
    n_rows = _check_rows(x, index, perm, base, n_rows)
    rows = x.index_select(0, _ref_rows(x.shape[0], n_rows, index, perm, base).to(x.device))
    out_dtype = out_dtype or x.dtype
    if out_dtype == x.dtype:
        return tuple(p.contiguous() for p in torch.split(rows, list(splits), dim=1))
    return tuple(p.float().to(out_dtype).contiguous() for p in torch.split(rows, list(splits), dim=1))


def split_columns(src, splits: Sequence[int], index: torch.Tensor | None = None, *,
                  perm: FeistelPermutation | None = None, base: int = 0, n_rows: int | None = None, out_dtype=None,
                  stream=None) -> tuple[torch.Tensor, ...]:
    """[N, nValues] rows -> tuple of contiguous [B, w_k] column groups (fused gather + cast)."""
    out_dtype = _dtypes.to_torch_dtype(out_dtype) if out_dtype is not None else src.dtype
    if src.dim() != 2:
        raise ValueError("split_columns expects [N, nValues]")
    if sum(splits) != src.shape[1]:
        raise ValueError("splits must sum to nValues")
    if not _is_gpu(src):
        return ref_split_columns(src, splits, index, perm, base, n_rows, out_dtype)
    if out_dtype != src.dtype and out_dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("split_columns casts to bf16 or f32 only (same-dtype splits are raw copies)")
    n_rows = _check_rows(src, index, perm, base, n_rows)
    # one allocation, k contiguous [n_rows, w] views (a caching-allocator call costs ~2.5 us of host time)
    buf = torch.empty(n_rows * sum(splits), dtype=out_dtype, device=src.device)
    outs, off = [], 0
    for w in splits:
        outs.append(buf[off:off + n_rows * w].view(n_rows, w))
        off += n_rows * w
    outs = tuple(outs)
    _native.hip().split_columns(
        dsts=[o.data_ptr() for o in outs], widths=[int(w) for w in splits], out_dt=_dtypes.code(out_dtype),
        src=_src_addr(src), in_dt=_dtypes.code(src.dtype), n_rows=n_rows, n_values=src.shape[1],
        stream=_stream_handle(stream), **_index_kw(index, perm, base))
    return outs


def ref_pack_columns(groups, index=None, perm=None, base=0, n_rows=None, out_dtype=None):
    g0 = groups[0]
    n_rows = _check_rows(g0, index, perm, base, n_rows)
    rows = _ref_rows(g0.shape[0], n_rows, index, perm, base).to(g0.device)
    out_dtype = out_dtype or g0.dtype
    cat = torch.cat([g.index_select(0, rows) for g in groups], dim=1)
    return cat if out_dtype == g0.dtype else cat.float().to(out_dtype)


def pack_columns(groups: Sequence[torch.Tensor], index: torch.Tensor | None = None, *,
                 perm: FeistelPermutation | None = None, base: int = 0, n_rows: int | None = None, out_dtype=None,
                 out: torch.Tensor | None = None, host_threads: int = 4, stream=None) -> torch.Tensor:
    """k [N, w_g] column groups -> one [B, sum w_g] row block.

    The reference fills each producer window by concatenating the harness's
    column groups on the host (tests/run_ddl.py:156-159). On the host this runs
    on the native thread pool (row-blocked memcpy, GIL released); on the GPU it
    is one gfx950 kernel fused with the row gather (index / Feistel perm) and
    the dtype cast -- the inverse of ``split_columns``.
    """
    groups = list(groups)
    if not 1 <= len(groups) <= 8:
        raise ValueError("pack_columns takes 1..8 groups")
    g0 = groups[0]
    for g in groups:
        if g.dim() != 2 or g.shape[0] != g0.shape[0] or g.dtype != g0.dtype or g.device != g0.device:
            raise ValueError("groups must be 2-D with equal row counts, dtype and device")
    widths = [int(g.shape[1]) for g in groups]
    n_values = sum(widths)
    out_dtype = _dtypes.to_torch_dtype(out_dtype) if out_dtype is not None else (
        out.dtype if out is not None else g0.dtype)
    n_rows = _check_rows(g0, index, perm, base, n_rows)
    if out is None:
        out = torch.empty((n_rows, n_values), dtype=out_dtype, device=g0.device)
    if tuple(out.shape) != (n_rows, n_values) or out.dtype != out_dtype or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous {(n_rows, n_values)} {out_dtype} tensor")
    groups = [g.contiguous() for g in groups]
    if not g0.is_cuda:
        if index is None and perm is None and out_dtype == g0.dtype:
            esz = g0.element_size()
            _native.runtime().pack_columns(out.data_ptr(), [g.data_ptr() + base * w * esz
                                                            for g, w in zip(groups, widths)],
                                           widths, esz, n_rows, host_threads)
            return out
        out.copy_(ref_pack_columns(groups, index, perm, base, n_rows, out_dtype))
        return out
    if out_dtype != g0.dtype and out_dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("pack_columns casts to bf16 or f32 only (same-dtype packs are raw copies)")
    if out.device != g0.device:
        raise ValueError("out must be on the groups' device")
    _native.hip().pack_columns(
        srcs=[g.data_ptr() for g in groups], widths=widths, in_dt=_dtypes.code(g0.dtype), dst=out.data_ptr(),
        out_dt=_dtypes.code(out_dtype), n_rows=n_rows, n_values=n_values, stream=_stream_handle(stream),
        **_index_kw(index, perm, base))
    return out


# --------------------------------------------------------------------- tokens
_TOK16 = (torch.int16, torch.uint16)


def widen_tokens(tokens: torch.Tensor) -> torch.Tensor:
    """int32 view of a token tensor: int32 as is; 2-byte tokens (uint16 ids on the wire, int16-typed views of
    them) zero-extended."""
    if tokens.dtype == torch.int32:
        return tokens
    if tokens.dtype == torch.int16:
        return tokens.to(torch.int32) & 0xFFFF
    if tokens.dtype == torch.uint16:
        return tokens.view(torch.int16).to(torch.int32) & 0xFFFF
    raise TypeError(f"tokens must be int32 or 16-bit, got {tokens.dtype}")


def ref_pad_tokens(tokens: torch.Tensor, offsets: torch.Tensor, seq_len: int, pad_id: int = 0,
                   position_dtype=torch.int64):
    offs = offsets.to("cpu", torch.int64).tolist()
    b = len(offs) - 1
    t = widen_tokens(tokens.cpu())
    out = torch.full((b, seq_len), pad_id, dtype=torch.int32)
    mask = torch.zeros((b, seq_len), dtype=torch.uint8)
    pos = torch.zeros((b, seq_len), dtype=position_dtype)
    for i in range(b):
        n = min(offs[i + 1] - offs[i], seq_len)
        if n > 0:
            out[i, :n] = t[offs[i]:offs[i] + n]
            mask[i, :n] = 1
            pos[i, :n] = torch.arange(n, dtype=position_dtype)
    return out, mask, pos


def pad_tokens(tokens: torch.Tensor, offsets: torch.Tensor, seq_len: int, pad_id: int = 0,
               position_dtype=torch.int64, stream=None):
    """Ragged token stream (int32, or 16-bit ids widened by the kernel) + [B+1] int64 offsets ->
    (tokens [B,S] i32, mask u8 [B,S], position ids [B,S])."""
    if (tokens.dtype != torch.int32 and tokens.dtype not in _TOK16) or offsets.dtype != torch.int64:
        raise TypeError("tokens must be int32 / 16-bit and offsets int64")
    if not tokens.is_cuda:
        return ref_pad_tokens(tokens, offsets, seq_len, pad_id, position_dtype)
    b = offsets.numel() - 1
    dev = tokens.device
    out = torch.empty((b, seq_len), dtype=torch.int32, device=dev)
    mask = torch.empty((b, seq_len), dtype=torch.uint8, device=dev)
    pos = torch.empty((b, seq_len), dtype=position_dtype, device=dev)
    _native.hip().pad_pack_tokens(
        tokens=tokens.data_ptr(), offsets=offsets.data_ptr(), row_start=0, row_end=0, seg_offsets=0, n_seg=0,
        out_tokens=out.data_ptr(), attn_mask=mask.data_ptr(), position_ids=pos.data_ptr(),
        pos_is_i64=position_dtype == torch.int64, segment_ids=0, cu_seqlens_out=0, rows=b, seq_len=seq_len,
        pad_id=pad_id, mode=0, stream=_stream_handle(stream), tok16=tokens.dtype in _TOK16)
    return out, mask, pos


def pack_plan(seq_offsets: np.ndarray, seq_len: int, max_rows: int | None = None):
    """Greedy in-order packing of sequences into rows of ``seq_len`` tokens (native C++).

    Sequences longer than ``seq_len`` are split into ``seq_len`` chunks (each
    chunk restarts its position ids). Returns (row_start, row_end, seg_offsets)
    int64 arrays: row r holds flat tokens [row_start[r], row_end[r]);
    seg_offsets are the (split) sequence starts plus the end. ``max_rows``
    truncates the plan (reference implementation).
    """
    offs = np.ascontiguousarray(seq_offsets, dtype=np.int64)
    if max_rows is not None:
        return ref_pack_plan(offs, seq_len, max_rows)
    n = len(offs) - 1
    lens = np.diff(offs)
    max_segs = int(np.sum(-(-lens // seq_len))) if n > 0 else 0
    rs = np.empty(max(max_segs, 1), np.int64)
    re_ = np.empty(max(max_segs, 1), np.int64)
    so = np.empty(max_segs + 1, np.int64)
    n_rows, n_seg = _native.runtime().pack_plan(offs.ctypes.data, n, int(seq_len), rs.ctypes.data, re_.ctypes.data,
                                               max(max_segs, 1), so.ctypes.data, max_segs)
    return rs[:n_rows].copy(), re_[:n_rows].copy(), so[: n_seg + 1].copy()


def ref_pack_plan(seq_offsets: np.ndarray, seq_len: int, max_rows: int | None = None):
    """Pure-Python reference of ``pack_plan``.

    Sequences longer than ``seq_len`` are split into ``seq_len`` chunks (each
    chunk restarts its position ids). Returns (row_start, row_end, seg_offsets)
    int64 arrays: row r holds flat tokens [row_start[r], row_end[r]);
    seg_offsets are the (split) sequence starts plus the end.
    """
    offs = np.asarray(seq_offsets, dtype=np.int64)
    segs = []
    for i in range(len(offs) - 1):
        s, e = int(offs[i]), int(offs[i + 1])
        while e - s > seq_len:
            segs.append((s, s + seq_len))
            s += seq_len
        if e > s:
            segs.append((s, e))
    row_start, row_end = [], []
    cur_s, cur_e = None, None
    for s, e in segs:
        if cur_s is None:
            cur_s, cur_e = s, e
        elif e - cur_s <= seq_len and s == cur_e:
            cur_e = e
        else:
            row_start.append(cur_s)
            row_end.append(cur_e)
            cur_s, cur_e = s, e
        if max_rows is not None and len(row_start) >= max_rows:
            break
    if cur_s is not None and (max_rows is None or len(row_start) < max_rows):
        row_start.append(cur_s)
        row_end.append(cur_e)
    seg_offsets = np.array([s for s, _ in segs] + ([segs[-1][1]] if segs else [0]), dtype=np.int64)
    return np.array(row_start, dtype=np.int64), np.array(row_end, dtype=np.int64), seg_offsets


def ref_pack_tokens(tokens, row_start, row_end, seg_offsets, seq_len, pad_id=0, position_dtype=torch.int64,
                    fill_rows: int = 0):
    """CPU reference of pack mode; ``fill_rows`` > packed rows: padding rows up to that fixed row count."""
    t = widen_tokens(tokens.cpu())
    rs, re_, so = (np.asarray(a) for a in (row_start, row_end, seg_offsets))
    r = max(len(rs), int(fill_rows))
    out = torch.full((r, seq_len), pad_id, dtype=torch.int32)
    mask = torch.zeros((r, seq_len), dtype=torch.uint8)
    pos = torch.zeros((r, seq_len), dtype=position_dtype)
    seg = torch.full((r, seq_len), -1, dtype=torch.int32)
    for i in range(len(rs)):
        n = min(int(re_[i] - rs[i]), seq_len)
        g = np.arange(rs[i], rs[i] + n)
        sidx = np.searchsorted(so, g, side="right") - 1
        out[i, :n] = t[rs[i]:rs[i] + n]
        mask[i, :n] = 1
        pos[i, :n] = torch.from_numpy(g - so[sidx]).to(position_dtype)
        seg[i, :n] = torch.from_numpy(sidx.astype(np.int32))
    return out, mask, pos, seg


def pack_capacity(n_seq: int, n_tokens: int, seq_len: int) -> tuple[int, int]:
    """(max segments, max rows) that in-order packing of ``n_seq`` sequences holding at most ``n_tokens``
    tokens can produce: each sequence splits into ceil(len / S) segments (<= n_seq + n_tokens // S in total),
    and two consecutive rows together hold more than S tokens (else the greedy pass would have merged them),
    so rows <= 2 * ceil(n_tokens / S) + 1."""
    S = int(seq_len)
    max_segs = int(n_seq) + int(n_tokens) // S
    max_rows = min(max_segs, 2 * (-(-int(n_tokens) // S)) + 1)
    return max_segs, max(max_rows, 0)


def pack_tokens_device(tokens: torch.Tensor, offsets: torch.Tensor, seq_len: int, pad_id: int = 0,
                       position_dtype=torch.int64, max_rows: int | None = None, stream=None) -> dict:
    """Pack with the plan built ON THE DEVICE: two launches (``pack_plan_device``, then the pack kernel
    reading the plan's row count from device memory), no host round trip, static output shapes.

    ``offsets`` is the [B+1] int64 offsets tensor on the tokens' device. Outputs have ``max_rows`` rows
    (default: ``pack_capacity`` of the token buffer, an upper bound the plan cannot exceed); rows past the
    plan's are padding (pad_id, mask 0, position 0, segment -1). Returns a dict: ``input_ids``,
    ``attention_mask``, ``position_ids``, ``segment_ids``, ``cu_seqlens`` (int32, capacity max_segs + 1; only
    the first n_seg + 1 entries are written), ``counts`` (device int64 [n_rows, n_seg]; n_rows = -1 if max_rows
    was too small, every row then padding). Reference of the plan: ``pack_plan`` (host, runtime/arena.cpp).
    Graph-capturable: nothing in it synchronises with the host.
    """
    if (tokens.dtype != torch.int32 and tokens.dtype not in _TOK16) or offsets.dtype != torch.int64:
        raise TypeError("tokens must be int32 / 16-bit and offsets int64")
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets needs at least one entry")
    S = int(seq_len)
    max_segs, cap_rows = pack_capacity(n, tokens.numel(), S)
    R = cap_rows if max_rows is None else int(max_rows)
    dev = tokens.device
    if not tokens.is_cuda:  # host reference: the same outputs from the host plan
        rs, re_, so = ref_pack_plan(offsets.cpu().numpy(), S)
        ok = len(rs) <= R
        out, mask, pos, seg = ref_pack_tokens(tokens, rs[:R] if ok else rs[:0], re_[:R] if ok else re_[:0], so, S,
                                              pad_id, position_dtype, fill_rows=R)
        cu = torch.zeros(max_segs + 1, dtype=torch.int32)
        cu[:len(so)] = torch.from_numpy(so.astype(np.int32))
        counts = torch.tensor([len(rs) if ok else -1, len(so) - 1], dtype=torch.int64)
        return {"input_ids": out[:R], "attention_mask": mask[:R], "position_ids": pos[:R], "segment_ids": seg[:R],
                "cu_seqlens": cu, "counts": counts}
    if not offsets.is_cuda or offsets.device != dev:
        raise ValueError("offsets must be on the tokens' device (use pack_tokens for host offsets)")
    h = _native.hip()
    offsets = offsets.contiguous()
    # one allocation for the plan, its scratch and the five outputs (16-byte aligned regions)
    pb = 8 if position_dtype == torch.int64 else 4
    sizes = [8 * (max_segs + 1), 8 * max(R, 1), 8 * max(R, 1), 16, 4 * h.pack_plan_scratch_ints(max_segs, R),
             4 * R * S, R * S, pb * R * S, 4 * R * S, 4 * (max_segs + 1)]
    offs_b = [0]
    for n_b in sizes:
        offs_b.append(offs_b[-1] + -(-n_b // 16) * 16)
    whole = torch.empty(offs_b[-1], dtype=torch.uint8, device=dev)
    reg = [whole[a:a + n_b] for a, n_b in zip(offs_b, sizes)]
    so, rs, re_, counts = (r.view(torch.int64) for r in reg[:4])
    scratch = reg[4].view(torch.int32)
    out = reg[5].view(torch.int32).view(R, S)
    mask = reg[6].view(R, S)
    pos = reg[7].view(position_dtype).view(R, S)
    seg = reg[8].view(torch.int32).view(R, S)
    cu = reg[9].view(torch.int32)
    sh = _stream_handle(stream)
    h.pack_plan_device(offsets=offsets.data_ptr(), n=n, seq_len=S, max_segs=max_segs, max_rows=R,
                       seg_offsets=so.data_ptr(), row_start=rs.data_ptr(), row_end=re_.data_ptr(),
                       counts=counts.data_ptr(), scratch=scratch.data_ptr(), stream=sh)
    if R > 0:
        h.pad_pack_tokens(
            tokens=tokens.data_ptr(), offsets=0, row_start=rs.data_ptr(), row_end=re_.data_ptr(),
            seg_offsets=so.data_ptr(), n_seg=0, out_tokens=out.data_ptr(), attn_mask=mask.data_ptr(),
            position_ids=pos.data_ptr(), pos_is_i64=position_dtype == torch.int64, segment_ids=seg.data_ptr(),
            cu_seqlens_out=cu.data_ptr(), rows=0, seq_len=S, pad_id=pad_id, mode=1, stream=sh, fill_rows=R,
            dev_counts=counts.data_ptr(), tok16=tokens.dtype in _TOK16)
    else:  # no rows to launch over: the (empty) plan's cu_seqlens is the single 0
        cu[:1].zero_()
    return {"input_ids": out, "attention_mask": mask, "position_ids": pos, "segment_ids": seg, "cu_seqlens": cu,
            "counts": counts}


def pack_tokens(tokens: torch.Tensor, seq_offsets, seq_len: int, pad_id: int = 0, position_dtype=torch.int64,
                stream=None):
    """Pack a ragged token stream into rows of ``seq_len`` (varlen-attention layout).

    Returns (tokens [R,S] i32, mask [R,S] u8, position_ids [R,S], segment_ids [R,S] i32 (-1 = pad),
    cu_seqlens [n_seg+1] i32 over the unpadded stream ``tokens[mask.bool()]``).

    Offsets already on the tokens' GPU: the plan is built on the device (``pack_tokens_device``) and the
    one host synchronisation is the read of the row count that sizes the result. Host offsets: the host
    plan (native ``pack_plan``), uploaded with the launch.
    """
    if tokens.is_cuda and torch.is_tensor(seq_offsets) and seq_offsets.device == tokens.device:
        r = pack_tokens_device(tokens, seq_offsets.to(torch.int64), seq_len, pad_id, position_dtype, stream=stream)
        n_rows, n_seg = (int(v) for v in r["counts"].cpu())
        if n_rows < 0:  # cannot happen within pack_capacity; kept loud
            raise RuntimeError(f"device pack plan overflowed ({n_seg} segments)")
        return (r["input_ids"][:n_rows], r["attention_mask"][:n_rows], r["position_ids"][:n_rows],
                r["segment_ids"][:n_rows], r["cu_seqlens"][:n_seg + 1])
    rs, re_, so = pack_plan(np.asarray(seq_offsets.cpu() if torch.is_tensor(seq_offsets) else seq_offsets),
                            seq_len)
    cu = torch.from_numpy(so.astype(np.int32))
    if not tokens.is_cuda:
        return (*ref_pack_tokens(tokens, rs, re_, so, seq_len, pad_id, position_dtype), cu)
    dev = tokens.device
    rs_d, re_d, so_d = (torch.from_numpy(a).to(dev, non_blocking=False) for a in (rs, re_, so))
    r = len(rs)
    out = torch.empty((r, seq_len), dtype=torch.int32, device=dev)
    mask = torch.empty((r, seq_len), dtype=torch.uint8, device=dev)
    pos = torch.empty((r, seq_len), dtype=position_dtype, device=dev)
    seg = torch.empty((r, seq_len), dtype=torch.int32, device=dev)
    _native.hip().pad_pack_tokens(
        tokens=tokens.data_ptr(), offsets=0, row_start=rs_d.data_ptr(), row_end=re_d.data_ptr(),
        seg_offsets=so_d.data_ptr(), n_seg=len(so) - 1, out_tokens=out.data_ptr(), attn_mask=mask.data_ptr(),
        position_ids=pos.data_ptr(), pos_is_i64=position_dtype == torch.int64, segment_ids=seg.data_ptr(),
        cu_seqlens_out=0, rows=r, seq_len=seq_len, pad_id=pad_id, mode=1, stream=_stream_handle(stream),
        tok16=tokens.dtype in _TOK16)
    return out, mask, pos, seg, so_d.to(torch.int32)


# ----------------------------------------------------------------- reductions
def ref_checksum(x: torch.Tensor) -> int:
    b = x.detach().contiguous().reshape(-1).view(torch.uint8).cpu().numpy()
    n = b.size // 4 * 4
    return int(b[:n].view(np.uint32).astype(np.uint64).sum()) & ((1 << 64) - 1)


def checksum(x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Sum of the 32-bit words of ``x`` (u64 wrap-around) as a 1-element int64 tensor (accumulates into ``out``)."""
    if not x.is_contiguous():
        raise ValueError("checksum needs a contiguous tensor")
    nbytes = x.numel() * x.element_size()
    if not x.is_cuda:
        v = ref_checksum(x)
        v = v - (1 << 64) if v >= (1 << 63) else v
        res = torch.tensor([v], dtype=torch.int64)
        if out is not None:
            out += res
            return out
        return res
    if out is None:
        out = torch.zeros(1, dtype=torch.int64, device=x.device)
    h = _native.hip()
    scratch = torch.empty(h.CHECKSUM_MAX_BLOCKS, dtype=torch.int64, device=x.device)
    h.checksum_words(ptr=x.data_ptr(), bytes=nbytes - nbytes % 4, out=out.data_ptr(), scratch=scratch.data_ptr(),
                     scratch_len=scratch.numel(), stream=_stream_handle(stream))
    return out


class ChecksumAccumulator:
    """Running checksum of many tensors: one streaming launch per ``add``.

    Each of ``n_partials`` workgroups adds its share of every tensor into its own
    64-bit slot (single writer, stream-ordered, no atomics); ``value()`` reduces
    the slots. Same sum as ``checksum`` (u64 wrap-around of the 32-bit words).
    Launches on one accumulator must be ordered on one stream.
    """

    def __init__(self, device, n_partials: int = 1024):
        self.device = torch.device(device)
        self.n = int(n_partials)
        self.partials = torch.zeros(self.n, dtype=torch.int64, device=self.device) if self.device.type == "cuda" \
            else None
        self._cpu = 0

    def add(self, x: torch.Tensor, stream=None) -> None:
        if not x.is_contiguous():
            raise ValueError("checksum needs a contiguous tensor")
        nbytes = x.numel() * x.element_size()
        if self.partials is None or not x.is_cuda:
            self._cpu = (self._cpu + ref_checksum(x)) & ((1 << 64) - 1)
            return
        if x.device != self.device:
            raise ValueError(f"tensor on {x.device}, accumulator on {self.device}")
        _native.hip().checksum_accumulate(ptr=x.data_ptr(), bytes=nbytes - nbytes % 4,
                                          partials=self.partials.data_ptr(), n_partials=self.n,
                                          stream=_stream_handle(stream))

    def value(self, stream=None) -> int:
        """Sum so far as an unsigned 64-bit int (synchronises with the accumulating stream)."""
        tot = self._cpu
        if self.partials is not None:
            out = torch.zeros(1, dtype=torch.int64, device=self.device)
            _native.hip().checksum_finalize(partials=self.partials.data_ptr(), n_partials=self.n,
                                            out=out.data_ptr(), stream=_stream_handle(stream))
            tot += int(out.item())
        return tot & ((1 << 64) - 1)


def column_affine(stats: dict, mode: str = "standard", area_weighted: bool = False) -> tuple[list, list]:
    """(scale, bias) per column so that x*scale + bias normalises like the reference harness.

    ``standard``: (x - mean) / std. ``minmax``: (x - (max+min)/2) / ((max-min)/2).
    ``area_weighted`` keeps the last column un-centred and scales it by its mean
    (reference tests/run_ddl.py:45-77).
    """
    mean, std, mn, mx = (stats[k].double().cpu() for k in ("mean", "std", "min", "max"))
    if mode == "standard":
        centre, spread = mean.clone(), std.clone()
    elif mode == "minmax":
        centre, spread = 0.5 * (mx + mn), 0.5 * (mx - mn)
    else:
        raise ValueError("mode must be 'standard' or 'minmax'")
    if area_weighted:
        centre[-1], spread[-1] = 0.0, mean[-1]
    spread = torch.where(spread == 0, torch.ones_like(spread), spread)
    return (1.0 / spread).tolist(), (-centre / spread).tolist()


def normalize_columns(x: torch.Tensor, mode: str = "standard", out_dtype=None, stats: dict | None = None,
                      area_weighted: bool = False, stream=None) -> torch.Tensor:
    """Per-column normalisation of an [N, C<=16] f32 table on the device (column_stats + fused affine gather)."""
    if x.dim() != 2 or x.shape[1] > 16:
        raise ValueError("normalize_columns expects [N, C] with C <= 16")
    stats = stats or column_stats(x, stream=stream)
    sc, bi = column_affine(stats, mode, area_weighted)
    return gather_rows(x, out_dtype=out_dtype or torch.float32, scale=sc, bias=bi, plane=1, stream=stream)


def column_stats(x: torch.Tensor, stream=None) -> dict[str, torch.Tensor]:
    """Per-column sum / sumsq / min / max / mean / std of an [N, C] f32 matrix."""
    if x.dim() != 2 or x.dtype != torch.float32:
        raise TypeError("column_stats expects [N, C] float32")
    n, c = x.shape
    if not x.is_cuda:
        s, q = x.double().sum(0).float(), (x.double() ** 2).sum(0).float()
        mn, mx = x.min(0).values, x.max(0).values
    else:
        x = x.contiguous()
        s = torch.zeros(c, dtype=torch.float32, device=x.device)
        q = torch.zeros_like(s)
        mn = torch.full_like(s, float("inf"))
        mx = torch.full_like(s, float("-inf"))
        _native.hip().column_stats(src=x.data_ptr(), n=n, cols=c, sum=s.data_ptr(), sumsq=q.data_ptr(),
                                   min=mn.data_ptr(), max=mx.data_ptr(), stream=_stream_handle(stream))
    mean = s / n
    var = (q / n - mean * mean).clamp_min(0)
    return {"sum": s, "sumsq": q, "min": mn, "max": mx, "mean": mean, "std": var.sqrt()}
