"""Counter-based, world-size-invariant epoch permutations.

``FeistelPermutation(n, seed, epoch)`` is a bijection of ``[0, n)`` computed
position-by-position by a 6-round balanced Feistel network with cycle walking
-- bit-identical to the device implementation in ``csrc/kernels/common.h``
(``feistel_perm``), which the gather kernels evaluate inline. No permutation
table is materialised or communicated; any rank can evaluate any position.

``EpochOrder`` turns it into the loader's global sample order: epoch ``e``
visits ``perm_e(0), perm_e(1), ...``; global batch ``g`` is positions
``[g*GB, (g+1)*GB)`` and DP rank ``r`` of ``W`` takes the contiguous slice
``[r*GB/W, (r+1)*GB/W)`` of it. The union over ranks of every global batch is
therefore the same for W = 1, 2, 4, 8 (BASELINE north star), and
a checkpoint is just ``(seed, epoch, global_batch_cursor)``.

This replaces the reference's rank-seeded per-producer ``rng.shuffle``
(reference tests/run_ddl.py:122,163-167), whose order depends on the rank
layout.
"""

from __future__ import annotations

import dataclasses
import functools

import numpy as np

ROUNDS = 6
_MASK64 = (1 << 64) - 1
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_S30, _S27, _S31 = np.uint64(30), np.uint64(27), np.uint64(31)


def _mix64_int(z: int) -> int:
    z &= _MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def _mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> _S30)) * _M1
        z = (z ^ (z >> _S27)) * _M2
    return z ^ (z >> _S31)


@functools.lru_cache(maxsize=4096)
def _round_keys_cached(seed: int, epoch: int) -> tuple[int, ...]:
    keys = []
    for r in range(ROUNDS):
        z = (seed * 0x9E3779B97F4A7C15 + epoch * 0xD1B54A32D192ED03 + (r + 1) * 0x8CB92BA72F3D8DD7) & _MASK64
        keys.append(_mix64_int(z))
    return tuple(keys)


def round_keys(seed: int, epoch: int) -> list[int]:
    """Derive the 6 Feistel round keys of (seed, epoch)."""
    return list(_round_keys_cached(int(seed), int(epoch)))


def half_bits_for(n: int) -> int:
    if n <= 0:
        raise ValueError("permutation domain must be positive")
    return max(1, ((n - 1).bit_length() + 1) // 2)


@dataclasses.dataclass(frozen=True)
class FeistelPermutation:
    n: int
    seed: int = 0
    epoch: int = 0

    @property
    def keys(self) -> list[int]:
        return round_keys(self.seed, self.epoch)

    @property
    def half_bits(self) -> int:
        return half_bits_for(self.n)

    def device_args(self) -> dict:
        """Arguments of the HIP kernels' RowIndex/FeistelKeys (mode 2)."""
        return {"keys": self.keys, "n_domain": self.n, "half_bits": self.half_bits}

    def _once(self, x: np.ndarray, keys: np.ndarray, h: int) -> np.ndarray:
        hb = np.uint64(h)
        mask = np.uint64((1 << h) - 1)
        left = x >> hb
        right = x & mask
        for k in keys:
            t = left ^ (_mix64(right ^ k) & mask)
            left = right
            right = t
        return (left << hb) | right

    def __call__(self, positions) -> np.ndarray:
        pos = np.ascontiguousarray(positions, dtype=np.int64)
        rt = _native_runtime()
        if rt is not None:  # C++ (GIL released): ~100x faster than the numpy network below
            return rt.feistel(self.keys, self.half_bits, self.n, pos)
        return self.numpy_eval(pos)

    def numpy_eval(self, positions) -> np.ndarray:
        """Pure-numpy evaluation (reference for the native and device versions)."""
        pos = np.asarray(positions, dtype=np.int64)
        if pos.size and (pos.min() < 0 or pos.max() >= self.n):
            raise IndexError(f"positions out of range [0, {self.n})")
        keys = np.array(self.keys, dtype=np.uint64)
        h = self.half_bits
        n = np.uint64(self.n)
        x = self._once(pos.astype(np.uint64).ravel(), keys, h)
        bad = x >= n
        while bad.any():
            x[bad] = self._once(x[bad], keys, h)
            bad = x >= n
        return x.astype(np.int64).reshape(pos.shape)

    def full(self) -> np.ndarray:
        return self(np.arange(self.n, dtype=np.int64))


def _native_runtime():
    try:
        from . import _native

        return _native.runtime()
    except Exception:  # pragma: no cover - runtime not built
        return None


class IdentityOrder:
    """The unshuffled order with the ``FeistelPermutation`` call surface (``EpochOrder(shuffle=False)``)."""

    def __init__(self, n: int):
        self.n = int(n)

    def __call__(self, pos) -> np.ndarray:
        pos = np.asarray(pos, dtype=np.int64)
        if pos.size and (pos.min() < 0 or pos.max() >= self.n):
            raise IndexError(f"positions out of range [0, {self.n})")
        return pos

    def full(self) -> np.ndarray:
        return np.arange(self.n, dtype=np.int64)


@dataclasses.dataclass
class EpochOrder:
    """Global sample order for DP training, invariant to the world size."""

    n_samples: int
    global_batch: int
    seed: int = 0
    drop_last: bool = True
    shuffle: bool = True  # False: positions in dataset order (evaluation), same batching and checkpoints

    def __post_init__(self) -> None:
        if self.global_batch <= 0 or self.n_samples <= 0:
            raise ValueError("n_samples and global_batch must be positive")
        if self.drop_last and self.n_samples < self.global_batch:
            raise ValueError("fewer samples than one global batch with drop_last=True")

    @property
    def batches_per_epoch(self) -> int:
        if self.drop_last:
            return self.n_samples // self.global_batch
        return -(-self.n_samples // self.global_batch)

    def local_batch(self, world_size: int) -> int:
        if self.global_batch % world_size:
            raise ValueError(f"global batch {self.global_batch} not divisible by world size {world_size}")
        return self.global_batch // world_size

    def perm(self, epoch: int) -> FeistelPermutation | IdentityOrder:
        if not self.shuffle:
            return IdentityOrder(self.n_samples)
        return FeistelPermutation(self.n_samples, self.seed, epoch)

    def positions(self, g: int, rank: int, world_size: int) -> np.ndarray:
        """Positions of rank ``rank``'s slice of global batch ``g``. With ``drop_last=False`` the last,
        partial global batch is completed by wrapping around to the start of the epoch's order
        (``DistributedSampler``-style padding): every batch has ``global_batch`` samples, and the
        first ``batches_per_epoch * global_batch - n_samples`` samples of the epoch appear twice."""
        lb = self.local_batch(world_size)
        start = g * self.global_batch + rank * lb
        pos = np.arange(start, start + lb, dtype=np.int64)
        return pos % self.n_samples

    def indices(self, epoch: int, g: int, rank: int = 0, world_size: int = 1) -> np.ndarray:
        """Sample indices of rank ``rank``'s share of global batch ``g`` in ``epoch``."""
        return self.perm(epoch)(self.positions(g, rank, world_size))


def ids_digest(indices) -> int:
    """64-bit digest (signed, to fit a slot tag) of an ordered list of sample indices: producers of the
    indexed order publish it with every window; ``verify_order`` recomputes it on the consumer."""
    import hashlib

    raw = np.ascontiguousarray(np.asarray(indices, dtype=np.int64)).tobytes()
    return int.from_bytes(hashlib.blake2b(raw, digest_size=8).digest(), "little", signed=True)


def batch_cursor(sd: dict, global_batch) -> int:
    """The global-batch cursor of an indexed checkpoint: ``global_batch_cursor``, or derived from
    ``global_sample_cursor`` (epoch/sample-index checkpoints) when only that is given."""
    if "global_batch_cursor" in sd:
        return int(sd["global_batch_cursor"])
    if "global_sample_cursor" not in sd:
        raise KeyError("indexed checkpoint without global_batch_cursor / global_sample_cursor")
    gb = int(global_batch or 0)
    sc = int(sd["global_sample_cursor"])
    if gb <= 0 or sc % gb:
        raise ValueError(f"global_sample_cursor={sc} is not a multiple of the global batch {gb}")
    return sc // gb
