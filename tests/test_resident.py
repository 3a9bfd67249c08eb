"""HBM-resident sharded loader with exact global shuffle (BASELINE configs 3/5), gloo on CPU."""

import numpy as np
import pytest
import torch

from tests.mp_harness import run_ranks


def _resident_rank(rank, world, name, n, gb, epochs, depth, resume=None, stop=None, replicate=False):
    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    src = SharedArraySource(name, n, (3,), "int64")
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ResidentGlobalLoader(src, gb, env, seed=11, depth=depth, n_epochs=epochs, resume_state=resume,
                                  replicate=replicate)
        if dl.replicated:  # the whole dataset (plus <= W-1 padding rows) on every rank, bit-exact
            assert dl.shard.shape[0] >= max(n, dl.S * world)
            assert torch.equal(dl.shard[:n], src.tensor())
        else:
            assert dl.shard.shape[0] == dl.hi - dl.lo
        out = []
        while dl.epoch < epochs:
            e = dl.epoch
            rows = []
            for i, b in enumerate(dl):
                assert b.shape == (gb // world, 3)
                rows.append(b[:, 0].clone())
                if stop is not None and (e, i) == stop:
                    sd = dl.state_dict()
                    return out, sd, dl.stats()
            out.append(torch.cat(rows).numpy())
        return out, None, dl.stats()


@pytest.fixture
def src():
    from ddl_amd.models import SharedArraySource

    n = 777
    data = torch.stack([torch.arange(n), -torch.arange(n), torch.arange(n) * 2], 1)
    s = SharedArraySource.create(f"ddl_amd_res_{np.random.randint(1 << 30)}", data)
    yield s
    s.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("replicate", [False, True])
@pytest.mark.parametrize("world,depth", [(1, 1), (2, 2), (3, 3), (4, 2), (8, 2)])
def test_resident_exact_global_order(src, world, depth, replicate):
    """Sharded (per-step all-to-all) and replicated (all-gather bring-up, no per-step collective) deliver the
    identical union order -- global batch g of the epoch permutation -- at W = 1..8: every sample exactly
    once per epoch."""
    from ddl_amd.permutation import EpochOrder

    gb = 48
    res = run_ranks(_resident_rank, world, src.name, src.n, gb, 2, depth, None, None, replicate, timeout=280)
    order = EpochOrder(src.n, gb, 11)
    bpe = order.batches_per_epoch
    for e in range(2):
        ref = order.perm(e).full()[: bpe * gb].reshape(bpe, gb)
        merged = np.concatenate([r[0][e].reshape(bpe, gb // world) for r in res], axis=1)
        assert np.array_equal(merged, ref)
        assert len(np.unique(merged)) == merged.size  # exactly once
    st = [r[2] for r in res]
    if world > 1 and not replicate:
        assert sum(s_["bytes_exchanged"] for s_ in st) > 0
    if world > 1 and replicate:  # the per-step traffic is gone; the bring-up moved (W-1)/W of the data
        assert all(s_["replicated"] and s_["bytes_exchanged"] == 0 for s_ in st)
        assert all(s_["bytes_replicated"] >= (world - 1) * (src.n // world) * 24 for s_ in st)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("save,resume", [((2, False), (1, False)), ((8, True), (2, False)), ((4, False), (8, True))])
def test_resident_resume_across_world_sizes(src, save, resume):
    """A checkpoint taken at one (W, mode) resumes at another: sharded <-> replicated, 1 <-> 8 ranks."""
    from ddl_amd.permutation import EpochOrder

    gb = 48
    (w0, rep0), (w1, rep1) = save, resume
    res = run_ranks(_resident_rank, w0, src.name, src.n, gb, 2, 2, None, (0, 3), rep0, timeout=280)
    sd = res[0][1]
    assert sd["global_batch_cursor"] == 4 and all(r[1] == sd for r in res)
    out = run_ranks(_resident_rank, w1, src.name, src.n, gb, 2, 1, sd, None, rep1, timeout=280)
    order = EpochOrder(src.n, gb, 11)
    bpe = order.batches_per_epoch
    for e, first in ((0, 4), (1, 0)):
        merged = np.concatenate([r[0][e].reshape(-1, gb // w1) for r in out], axis=1).reshape(-1)
        assert np.array_equal(merged, order.perm(e).full()[first * gb: bpe * gb])


def _scatter_rank(rank, world, name, n, gb, replicate=False):
    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    src = SharedArraySource(name, n, (3,), "int64") if rank == 0 else None
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ResidentGlobalLoader(src, gb, env, seed=11, n_epochs=1, scatter_from=0, chunk_bytes=24 * 50,
                                  replicate=replicate)
        shard = dl.shard[:n].clone() if dl.replicated else dl.shard.clone()
        rows = torch.cat([b[:, 0].clone() for b in dl]).numpy()
        lo, hi = (0, n) if dl.replicated else (dl.lo, dl.hi)
        st = dl.stats()
        return shard.numpy(), rows, lo, hi, st["bytes_exchanged"] + st["bytes_replicated"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("replicate", [False, True])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_resident_scatter_from_one_rank(src, world, replicate):
    from ddl_amd.permutation import EpochOrder

    gb = 48
    res = run_ranks(_scatter_rank, world, src.name, src.n, gb, replicate, timeout=280)
    full = src.tensor().numpy()
    for shard, _, lo, hi, _ in res:
        assert np.array_equal(shard, full[lo:hi])  # every rank received exactly its shard (or the whole set)
    order = EpochOrder(src.n, gb, 11)
    bpe = order.batches_per_epoch
    ref = order.perm(0).full()[: bpe * gb].reshape(bpe, gb)
    merged = np.concatenate([r[1].reshape(bpe, gb // world) for r in res], axis=1)
    assert np.array_equal(merged, ref)
    assert res[0][4] > 0


def _close_rank(rank, world, name, n, gb):
    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    src = SharedArraySource(name, n, (3,), "int64")
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ResidentGlobalLoader(src, gb, env, seed=11, depth=2)
        it = iter(dl)
        next(it)
        dl.close()  # releases the shard even though `it` still references the loader
        assert dl.shard is None and dl.stats()["shard_rows"] == dl.hi - dl.lo
        try:
            next(it)
        except RuntimeError as e:
            return "closed" in str(e)
        return False


def test_resident_close_releases_shard(src):
    assert run_ranks(_close_rank, 1, src.name, src.n, 48) == [True]


def test_resident_augment_needs_gpu_and_known_keys(src):
    from ddl_amd.resident import ResidentGlobalLoader

    with pytest.raises(ValueError, match="handoff"):
        ResidentGlobalLoader(src, 48, handoff="sideways", device="cpu")
    with pytest.raises(ValueError, match="replicate"):
        ResidentGlobalLoader(src, 48, replicate="sometimes", device="cpu")

    with pytest.raises(ValueError):
        ResidentGlobalLoader(src, 48, augment={"size": (4, 4)}, device="cpu")  # CPU, and rows are not images
    with pytest.raises(ValueError):
        ResidentGlobalLoader(src, 48, augment={"bogus": 1}, device="cpu")


def _resident_live_reload_rank(rank, world, name, n, gb):
    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    src = SharedArraySource(name, n, (3,), "int64")
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ResidentGlobalLoader(src, gb, env, seed=11, depth=2, n_epochs=3)
        full = [b[:, 0].clone() for e in range(3) for b in dl]
        dl.set_epoch(0)  # rewind the same loader: epoch 0 again, from its first batch
        head, sd = [], None
        for i, b in enumerate(dl):
            head.append(b[:, 0].clone())
            if i == 4:
                sd = dl.state_dict()
                break
        for _ in range(2):  # run on into epoch 1 (a stale iterator is abandoned mid-epoch)
            for b in dl:
                pass
        dl.load_state_dict(sd)
        tail = []
        while dl.epoch < 3:
            tail += [b[:, 0].clone() for b in dl]
        return torch.cat(full).numpy(), torch.cat(head + tail).numpy()


@pytest.mark.parametrize("world", [1, 2])
def test_resident_live_load_state_dict_and_set_epoch(src, world):
    for full, resumed in run_ranks(_resident_live_reload_rank, world, src.name, src.n, 48):
        assert np.array_equal(full, resumed)
