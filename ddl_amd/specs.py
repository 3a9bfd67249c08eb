"""Grouped options of ``DistributedDataLoader`` beyond the reference's eight arguments.

The reference constructor takes eight arguments (reference ddl/mpi_dataloader.py:108-118). The
MI355X-native loader adds output conversion, device staging and ordering; instead of ~20 more keywords
they come in three frozen records:

* :class:`OutputSpec` -- what a batch looks like: dtype, per-channel normalisation, on-device augmentation,
  token collate, contiguous column groups, owned copies vs window views;
* :class:`StagingSpec` -- how windows reach HBM: prefetch depth, slots per producer, timeouts, per-batch
  dispatch, run-ahead bound, producer host threads, copy timing;
* :class:`OrderSpec` -- which samples come in which order: window / indexed mode, device shuffle, seed,
  order verification.

Each record validates itself. The flat keywords of earlier releases (``out_dtype=``, ``prefetch_depth=``,
``seed=`` ...) are still accepted by the constructor as deprecated aliases (:func:`resolve`).
"""

from __future__ import annotations

import dataclasses
import warnings
from typing import Any

MODES = ("do_not_split_along_epoch", "split_along_epoch", "window", "indexed")
AUGMENT_KEYS = frozenset({"size", "scale", "ratio", "flip_p", "layout"})
DISPATCH = (True, False, "auto", "inline", "lookahead", "window")


@dataclasses.dataclass(frozen=True)
class OutputSpec:
    """What a batch looks like.

    ``dtype``: device output dtype (None: the window's); ``normalize``: ``{"mean", "std"[, "scale", "bias",
    "layout": "chw"|"hwc"]}`` per-channel affine fused into the gather; ``augment``: on-device
    RandomResizedCrop + flip ``{"size", "scale", "ratio", "flip_p", "layout"}`` (GPU only, normalize applies
    after it); ``collate="tokens"``: token windows -> ``input_ids`` / ``attention_mask`` / ``position_ids``
    (``pad_id``; ``token_rows="fixed"`` keeps every packed batch at the window's row count);
    ``contiguous``: own each column group; ``copy_batches``: batches are owned copies (default: with
    ``auto_mark``, since the caller does not control the window's release) instead of window views."""

    dtype: Any = None
    normalize: dict | None = None
    augment: dict | None = None
    collate: str | None = None
    contiguous: bool = False
    copy_batches: bool | None = None
    pad_id: int = 0
    token_rows: str = "exact"

    def __post_init__(self):
        if self.augment is not None and not set(self.augment) <= AUGMENT_KEYS:
            raise ValueError(f"unknown augment keys {sorted(set(self.augment) - AUGMENT_KEYS)}")
        if self.collate not in (None, "tokens"):
            raise ValueError("collate must be None or 'tokens'")
        if self.token_rows not in ("exact", "fixed"):
            raise ValueError("token_rows must be 'exact' or 'fixed'")


@dataclasses.dataclass(frozen=True)
class StagingSpec:
    """How windows reach HBM.

    ``prefetch_depth``: HBM ring depth in windows; ``n_slots``: windows per producer (None: the producer's
    ``preferred_slots``); ``timeout_s``: bound on every wait (None: the connection's); ``native_dispatch``:
    per-batch dispatch by the C++ engine (True / "auto" / "inline" / "lookahead" / "window") or the Python
    path (False); ``max_ahead``: run-ahead bound in batches (None: 16; 0 off); ``host_threads``: producer
    host threads; ``copy_timing``: device times of every window copy (process-wide ROCr switch)."""

    prefetch_depth: int = 4
    n_slots: int | None = None
    timeout_s: float | None = None
    native_dispatch: bool | str = True
    max_ahead: int | None = None
    host_threads: int = 4
    copy_timing: bool = False

    def __post_init__(self):
        if self.native_dispatch not in DISPATCH:
            raise ValueError("native_dispatch must be a bool or 'auto' / 'inline' / 'lookahead' / 'window'")
        if self.max_ahead is not None and self.max_ahead < 0:
            raise ValueError("max_ahead must be >= 0")
        if self.prefetch_depth < 1:
            raise ValueError("prefetch depth must be >= 1")


@dataclasses.dataclass(frozen=True)
class OrderSpec:
    """Which samples come in which order.

    ``mode``: "window" (= the reference's "do_not_split_along_epoch": an epoch is one producer window),
    "split_along_epoch" (an epoch is one window of every producer) or "indexed" (windows of the
    world-size-invariant epoch order from indexed producers); ``shuffle="device"``: a fresh Feistel order
    inside every window visit, evaluated in the gather kernel; ``seed``; ``verify``: check every indexed
    window against the epoch order (None: ``$DDL_VERIFY_ORDER``)."""

    mode: str = "window"
    shuffle: str = "none"
    seed: int = 0
    verify: bool | None = None

    def __post_init__(self):
        if self.mode not in MODES:
            raise ValueError(f"unknown mode {self.mode!r}; one of {MODES}")
        if self.shuffle not in ("none", "device"):
            raise ValueError("shuffle must be 'none' or 'device'")


# flat keyword of earlier releases -> (record, field)
LEGACY: dict[str, tuple[str, str]] = {
    "out_dtype": ("output", "dtype"), "normalize": ("output", "normalize"), "augment": ("output", "augment"),
    "collate": ("output", "collate"), "contiguous": ("output", "contiguous"),
    "copy_batches": ("output", "copy_batches"), "pad_id": ("output", "pad_id"),
    "token_rows": ("output", "token_rows"),
    "prefetch_depth": ("staging", "prefetch_depth"), "n_slots": ("staging", "n_slots"),
    "timeout_s": ("staging", "timeout_s"), "native_dispatch": ("staging", "native_dispatch"),
    "max_ahead": ("staging", "max_ahead"), "host_threads": ("staging", "host_threads"),
    "copy_timing": ("staging", "copy_timing"),
    "mode": ("order", "mode"), "shuffle": ("order", "shuffle"), "seed": ("order", "seed"),
    "verify_order": ("order", "verify"),
}


def resolve(output: OutputSpec | None, staging: StagingSpec | None, order: OrderSpec | None,
            legacy: dict) -> tuple[OutputSpec, StagingSpec, OrderSpec]:
    """The three records, with any flat legacy keyword folded in (a ``DeprecationWarning`` names its new
    home). A keyword the loader never had is a ``TypeError``, as for any function."""
    unknown = sorted(set(legacy) - set(LEGACY))
    if unknown:
        raise TypeError(f"DistributedDataLoader() got unexpected keyword argument(s) {unknown}")
    groups: dict[str, dict] = {"output": {}, "staging": {}, "order": {}}
    for k, v in legacy.items():
        rec, field = LEGACY[k]
        groups[rec][field] = v
        warnings.warn(f"DistributedDataLoader({k}=...) is deprecated: use {rec}="
                      f"{rec.capitalize() if rec != 'output' else 'Output'}Spec({field}=...)",
                      DeprecationWarning, stacklevel=4)  # resolve <- __init__ <- with_logging <- caller
    out = dataclasses.replace(output or OutputSpec(), **groups["output"])
    stg = dataclasses.replace(staging or StagingSpec(), **groups["staging"])
    odr = dataclasses.replace(order or OrderSpec(), **groups["order"])
    return out, stg, odr


def from_flat(kw: dict, **order: Any) -> dict:
    """``{"output", "staging", "order"}`` records built from flat loader keywords ``kw`` (consumed from it) --
    for wrappers whose own signature forwards flat loader options (``ddl_amd.DataLoader(**loader_kw)``),
    without the deprecation warning; ``order`` sets OrderSpec fields the wrapper fixes itself."""
    groups: dict[str, dict] = {"output": {}, "staging": {}, "order": dict(order)}
    for k in [k for k in kw if k in LEGACY]:
        rec, field = LEGACY[k]
        groups[rec][field] = kw.pop(k)
    return {"output": OutputSpec(**groups["output"]), "staging": StagingSpec(**groups["staging"]),
            "order": OrderSpec(**groups["order"])}
