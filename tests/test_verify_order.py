"""``verify_order``: every window of the indexed order is checked against ``EpochOrder`` on the consumer
(slot tags = epoch, global batch, digest of the sample ids, published by ``IndexedProducer``).
SURVEY §5 race detection: a debug mode comparing delivered sample ids with the expected permutation."""

import numpy as np
import pytest
import torch

import ddl_amd
from ddl_amd.exceptions import DataIntegrityError
from ddl_amd.models import IndexedProducer, SharedArraySource
from ddl_amd.permutation import EpochOrder, ids_digest
from tests.mp_harness import run_ranks


@pytest.fixture
def source():
    n = 640
    data = torch.stack([torch.arange(n), torch.arange(n) * 3], 1)
    src = SharedArraySource.create(f"ddl_amd_vsrc_{np.random.randint(1 << 30)}", data)
    yield src
    src.close()


class SkewedProducer(IndexedProducer):
    """Delivers global batch g+1 where g is due, from round 1 on (a cursor bug), with honest tags.
    With 2 producers, round 1 of producer 0 is window 2."""

    def batch_position(self, rnd):
        epoch, g = super().batch_position(rnd)
        return (epoch, (g + 1) % self.order.batches_per_epoch) if rnd >= 1 else (epoch, g)


def _run(src, gb, epochs, producer_cls=IndexedProducer, resume=None, stop_after=None, verify=True):
    out = []
    with ddl_amd.start(n_producers=2, device="cpu") as (env, conn):
        dl = ddl_amd.DistributedDataLoader(producer_cls(src, gb, seed=3), gb // env.world_size, conn, epochs, env=env,
                                           auto_mark=True, resume_state=resume,
                                           order=ddl_amd.OrderSpec(mode="indexed", verify=verify))
        for e in range(dl.epoch, epochs):
            for i, (b,) in enumerate(dl):
                out.append(b[:, 0].clone())
                if stop_after is not None and (e, i + 1) == stop_after:
                    sd = dl.state_dict()
                    n = dl.verified_windows
                    dl.close()
                    return out, sd, n
        n = dl.stats().get("verified_windows", dl.verified_windows)
    return out, None, n


def test_digest_is_order_sensitive():
    a = np.arange(10)
    assert ids_digest(a) == ids_digest(a.copy()) and ids_digest(a) != ids_digest(a[::-1])


def test_every_window_is_verified(source, monkeypatch):
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    out, _, n = _run(source, 64, 2)
    order = EpochOrder(source.n, 64, 3)
    assert n == 2 * order.batches_per_epoch == len(out)
    assert torch.equal(out[0], torch.from_numpy(order.indices(0, 0)))


def test_skewed_producer_is_caught(source, monkeypatch):
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    with pytest.raises(DataIntegrityError, match="window 2: the epoch order expects \\(epoch 0, global batch 2"):
        _run(source, 64, 1, producer_cls=SkewedProducer)
    _run(source, 64, 1, producer_cls=SkewedProducer, verify=False)  # unverified: silently wrong samples


def test_resume_is_verified(source, monkeypatch):
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    _, sd, _ = _run(source, 64, 2, stop_after=(0, 4))
    out, _, n = _run(source, 64, 2, resume=sd)
    order = EpochOrder(source.n, 64, 3)
    assert n == len(out) == 2 * order.batches_per_epoch - 4


def test_window_mode_rejects_verify_order(monkeypatch):
    from tests.helpers import IdProducer

    monkeypatch.setenv("DDL_DEVICE", "cpu")
    with ddl_amd.start(n_producers=1, device="cpu") as (env, conn):
        with pytest.raises(ValueError, match="verify_order"):
            ddl_amd.DistributedDataLoader(IdProducer(16, 4), 8, conn, 1, env=env, order=ddl_amd.OrderSpec(verify=True))


def _rank(rank, world, name, n):
    src = SharedArraySource(name, n, (2,), "int64")
    out, _, nv = _run(src, 64, 1)
    return nv, len(out)


def test_verified_across_two_ranks(source):
    res = run_ranks(_rank, 2, source.name, source.n, env={"DDL_DEVICE": "cpu"})
    bpe = EpochOrder(source.n, 64, 3).batches_per_epoch
    assert all(nv == cnt == bpe for nv, cnt in res)


@pytest.mark.gpu
@pytest.mark.parametrize("native", [True, False])
def test_verify_order_on_device(source, native):
    """Staged windows (HBM ring): the native engine's slot tags and the Python stager's are checked."""
    bpe = EpochOrder(source.n, 64, 3).batches_per_epoch
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(source, 64, seed=3), 64, conn, 2, env=env, auto_mark=True,
                                           staging=ddl_amd.StagingSpec(native_dispatch=native),
                                           order=ddl_amd.OrderSpec(mode="indexed", verify=True))
        n = 0
        for _ in range(2):
            for (b,) in dl:
                assert b.is_cuda
                n += 1
        assert dl.verified_windows == n == 2 * bpe
        dl.close()
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(SkewedProducer(source, 64, seed=3), 64, conn, 1, env=env, auto_mark=True,
                                           staging=ddl_amd.StagingSpec(native_dispatch=native),
                                           order=ddl_amd.OrderSpec(mode="indexed", verify=True))
        with pytest.raises(DataIntegrityError):
            for _ in dl:
                pass
        dl.close()
