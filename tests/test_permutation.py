"""Counter-based permutation + world-size-invariant epoch order."""

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from ddl_amd.permutation import EpochOrder, FeistelPermutation, half_bits_for, round_keys

MASK = (1 << 64) - 1


def _mix(z):
    z &= MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def _py_perm(i, n, seed, epoch):
    """Independent scalar reference of csrc/kernels/common.h::feistel_perm."""
    keys = round_keys(seed, epoch)
    h = half_bits_for(n)
    mask = (1 << h) - 1

    def once(x):
        left, right = x >> h, x & mask
        for k in keys:
            left, right = right, left ^ (_mix(right ^ k) & mask)
        return (left << h) | right

    x = once(i)
    while x >= n:
        x = once(x)
    return x


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 1000, 4095, 4096, 4097, 100_520])
def test_bijection(n):
    p = FeistelPermutation(n, seed=1, epoch=2).full()
    assert np.array_equal(np.sort(p), np.arange(n))


@pytest.mark.parametrize("n", [1, 10, 1000, 65537])
def test_matches_scalar_reference(n):
    p = FeistelPermutation(n, seed=99, epoch=4)
    pos = np.unique(np.linspace(0, n - 1, num=min(n, 50)).astype(np.int64))
    assert [int(v) for v in p(pos)] == [_py_perm(int(i), n, 99, 4) for i in pos]


def test_deterministic_and_epoch_dependent():
    a = FeistelPermutation(10_000, 5, 0).full()
    b = FeistelPermutation(10_000, 5, 0).full()
    c = FeistelPermutation(10_000, 5, 1).full()
    d = FeistelPermutation(10_000, 6, 0).full()
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)
    assert not np.array_equal(a, d)
    # looks shuffled: few fixed points, low rank correlation
    assert (a == np.arange(10_000)).sum() < 50
    assert abs(np.corrcoef(a, np.arange(10_000))[0, 1]) < 0.05


def test_positions_out_of_range():
    p = FeistelPermutation(10)
    with pytest.raises(IndexError):
        p([10])
    with pytest.raises(IndexError):
        p([-1])


@settings(max_examples=60, deadline=None)
@given(n=st.integers(1, 5000), seed=st.integers(0, 2**63 - 1), epoch=st.integers(0, 10**6))
def test_bijection_property(n, seed, epoch):
    p = FeistelPermutation(n, seed, epoch).full()
    assert np.array_equal(np.sort(p), np.arange(n))


@pytest.mark.parametrize("n,gb", [(1000, 64), (100_520, 4096), (50, 8)])
def test_epoch_order_world_size_invariant(n, gb):
    order = EpochOrder(n, gb, seed=3)
    for epoch in (0, 1):
        for g in range(order.batches_per_epoch):
            ref = order.indices(epoch, g, 0, 1)
            for w in (2, 4, 8):
                if gb % w:
                    continue
                parts = [order.indices(epoch, g, r, w) for r in range(w)]
                assert np.array_equal(np.concatenate(parts), ref)


def test_epoch_order_exactly_once():
    order = EpochOrder(1000, 64, seed=1)
    for epoch in range(3):
        idx = np.concatenate([order.indices(epoch, g) for g in range(order.batches_per_epoch)])
        assert len(idx) == 15 * 64
        assert len(np.unique(idx)) == len(idx)
    order2 = EpochOrder(1000, 64, seed=1, drop_last=False)
    assert order2.batches_per_epoch == 16
    idx = np.concatenate([order2.indices(0, g) for g in range(16)])
    # the last global batch wraps around: every sample once, the epoch's first 24 twice, full batches
    assert len(idx) == 16 * 64 and np.array_equal(np.unique(idx), np.arange(1000))
    assert np.array_equal(idx[1000:], idx[:24])
    parts = [order2.indices(0, 15, r, 4) for r in range(4)]
    assert np.array_equal(np.concatenate(parts), idx[15 * 64:])


def test_epoch_order_validation():
    with pytest.raises(ValueError):
        EpochOrder(10, 64)
    with pytest.raises(ValueError):
        EpochOrder(1000, 64).local_batch(3)


@pytest.mark.parametrize("n", [1, 3, 1000, 1_281_167])
def test_native_matches_numpy_network(n):
    p = FeistelPermutation(n, seed=77, epoch=5)
    pos = np.unique(np.random.default_rng(0).integers(0, n, size=min(n, 3000)))
    assert np.array_equal(p(pos), p.numpy_eval(pos))
