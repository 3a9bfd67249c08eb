"""Multi-rank (DP) behaviour over gloo on CPU: world-size-invariant order, global
shuffle exchange, resume at a different world size (SURVEY §4.4 level 2)."""

import numpy as np
import pytest
import torch

from tests.mp_harness import run_ranks


def _indexed_rank(rank, world, n, gb, epochs, name, resume=None, stop_after=None):
    import ddl_amd
    from ddl_amd.models import IndexedProducer, SharedArraySource

    src = SharedArraySource(name, n, (2,), "int64")
    out = []
    with ddl_amd.start(n_producers=2) as (env, conn):
        assert env.world_size == world and env.rank == rank
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, gb, seed=7), gb // world, conn, epochs, env=env,
                                           auto_mark=True, resume_state=resume,
                                           order=ddl_amd.OrderSpec(mode="indexed"))
        for e in range(dl.epoch, epochs):
            rows = []
            for i, (b,) in enumerate(dl):
                rows.append(b[:, 0].clone())
                if stop_after is not None and e == stop_after[0] and i + 1 == stop_after[1]:
                    sd = dl.state_dict()
                    dl.close()
                    return out, sd
            out.append(torch.cat(rows).numpy())
    return out, None


@pytest.fixture
def shared_source():
    from ddl_amd.models import SharedArraySource

    n = 1000
    data = torch.stack([torch.arange(n), torch.arange(n) * 10], 1)
    src = SharedArraySource.create(f"ddl_amd_src_{np.random.randint(1 << 30)}", data)
    yield src
    src.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_indexed_order_is_world_size_invariant(shared_source, world):
    from ddl_amd.permutation import EpochOrder

    n, gb, epochs = shared_source.n, 64, 2
    res = run_ranks(_indexed_rank, world, n, gb, epochs, shared_source.name, timeout=280)
    order = EpochOrder(n, gb, seed=7)
    for e in range(epochs):
        ref = order.perm(e).full()[: order.batches_per_epoch * gb].reshape(-1, gb)
        per_rank = [r[0][e].reshape(-1, gb // world) for r in res]
        merged = np.concatenate(per_rank, axis=1)  # global batch g = concat of rank slices
        assert np.array_equal(merged, ref)
        assert len(np.unique(merged)) == merged.size  # exactly once per epoch


def test_indexed_resume_at_different_world_size(shared_source):
    n, gb = shared_source.n, 64
    # run on 2 ranks, stop after epoch 0 batch 5 (global batch cursor = 5)
    res = run_ranks(_indexed_rank, 2, n, gb, 2, shared_source.name, None, (0, 5))
    sd = res[0][1]
    assert sd["kind"] == "indexed" and sd["global_batch_cursor"] == 5 and sd["global_sample_cursor"] == 5 * gb
    sd = {k: v for k, v in sd.items() if k != "global_batch_cursor"}  # resume from the sample index alone
    # resume on 1 rank
    (out, _), = run_ranks(_indexed_rank, 1, n, gb, 2, shared_source.name, sd)
    from ddl_amd.permutation import EpochOrder

    order = EpochOrder(n, gb, seed=7)
    ref0 = order.perm(0).full()[5 * gb: order.batches_per_epoch * gb]
    assert np.array_equal(out[0], ref0)
    ref1 = order.perm(1).full()[: order.batches_per_epoch * gb]
    assert np.array_equal(out[1], ref1)


def _exchange_rank(rank, world, method, fraction, epochs=3):
    import ddl_amd
    from ddl_amd import Marker
    from tests.helpers import IdProducer

    eps = []
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(40, 6), 8, conn, epochs, fraction, method, env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           order=ddl_amd.OrderSpec(seed=1))
        assert dl._exchange_fn is not None
        for e in range(epochs):
            rows = []
            for i, (a, b) in enumerate(dl):
                rows.append(torch.cat([a, b], 1))
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
            eps.append(torch.cat(rows).numpy())
        n_ex = dl._exchange_fn.n_exchange
    return eps, n_ex


def _partner_cycles(n: int, seed: int, window: int) -> list[int]:
    """Cycle lengths of the sendrecv_replace partner permutation of ``window`` (send_to of every rank)."""
    from ddl_amd.parallel.shuffle import derangement_partners

    to = [derangement_partners(n, r, np.random.default_rng([seed & 0xFFFFFFFF, window]))[0] for r in range(n)]
    seen, out = set(), []
    for r in range(n):
        c, x = 0, r
        while x not in seen:
            seen.add(x)
            x, c = to[x], c + 1
        if c:
            out.append(c)
    return sorted(out)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("method,world", [("alltoall", 2), ("alltoall", 4), ("alltoall", 8), ("sendrecv_replace", 2),
                                          ("sendrecv_replace", 3), ("sendrecv_replace", 8)])
def test_global_shuffle_exchange_conserves_rows(method, world):
    """Exactly-once delivery across the exchange: every (rank, producer, row) key of every window is delivered
    once, by some rank, every epoch. At W = 8 the reference's partner rule can split the ranks into several
    cycles (5 + 3); the run covers such a window (window 3 with seed 1), where the reference's
    "prevents split graph" comment would have it deadlock or lose rows."""
    epochs = 4 if world == 8 else 3
    if method == "sendrecv_replace" and world == 8:
        assert _partner_cycles(8, 1, 3) == [3, 5]  # a split pattern among the exchanged windows
        assert _partner_cycles(8, 1, 0) == [8]
    res = run_ranks(_exchange_rank, world, method, 0.5, epochs, timeout=280)
    n_ex = res[0][1]
    assert n_ex > 0
    for e in range(epochs):
        all_rows = np.concatenate([r[0][e] for r in res])
        # every rank's window rows (rank, producer, i) are still delivered exactly once overall
        keys = {tuple(x) for x in all_rows[:, :3].tolist()}
        assert len(keys) == len(all_rows) == world * 40
        for r in range(world):
            mine = res[r][0][e]
            foreign = (mine[:, 0] != r).sum()
            if method == "alltoall":
                assert foreign == n_ex - n_ex // world  # chunk for self stays
            else:
                assert foreign == n_ex


def test_npy_memmap_source_indexed(tmp_path):
    import ddl_amd
    from ddl_amd.models import IndexedProducer, NpyMemmapSource
    from ddl_amd.permutation import EpochOrder

    arr = np.stack([np.arange(500), np.arange(500) * 2], 1).astype(np.int32)
    path = tmp_path / "data.npy"
    np.save(path, arr)
    src = NpyMemmapSource(str(path))
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, 50, seed=2), 50, conn, 1, env=env, auto_mark=True,
                                           order=ddl_amd.OrderSpec(mode="indexed"))
        got = torch.cat([b[0].cpu() for b in dl]).numpy()
    ref = EpochOrder(500, 50, 2).perm(0).full()
    assert np.array_equal(got[:, 0], ref) and np.array_equal(got[:, 1], ref * 2)


def _topology_rank(rank, world, method):
    import ddl_amd

    with ddl_amd.start(n_producers=1) as (env, conn):
        info = (env.hostname, env.node_rank, env.local_rank, env.local_world_size)
        from tests.helpers import IdProducer

        dl = ddl_amd.DistributedDataLoader(IdProducer(40, 4), 8, conn, 2, 0.5, method, env.rank, env.world_size,
                                           env=env, output=ddl_amd.OutputSpec(copy_batches=True))
        rows = []
        for _ in range(2):
            for b in dl:
                rows.append(torch.cat(b, 1).clone())
                dl.mark(ddl_amd.Marker.END_OF_BATCH)
            dl.mark(ddl_amd.Marker.END_OF_EPOCH)
    return info, torch.cat(rows).numpy()


@pytest.mark.parametrize("method", ["alltoall", "sendrecv_replace"])
def test_two_node_rehearsal(method):
    """2 "nodes" x 2 ranks (DDL_HOSTNAME per node): node ranks / local ranks come out right, the
    node-locality check passes, and the global-shuffle exchange spans both nodes."""
    res = run_ranks(_topology_rank, 4, method, nodes=2)
    infos = [r[0] for r in res]
    assert infos == [("rehearsal-node0", 0, 0, 2), ("rehearsal-node0", 0, 1, 2),
                     ("rehearsal-node1", 1, 0, 2), ("rehearsal-node1", 1, 1, 2)]
    rows = np.concatenate([r[1] for r in res])
    keys = {tuple(x) for x in rows[:, :4].tolist()}  # (rank, producer, i, round): exchanged, never duplicated
    assert len(keys) == len(rows) == 4 * 2 * 40
    foreign = [int((r[1][:, 0] != k).sum()) for k, r in enumerate(res)]
    assert all(f > 0 for f in foreign)  # every rank received rows from others (incl. the other node)


def _bad_topology_rank(rank, world):
    import ddl_amd

    with ddl_amd.start(n_producers=0):
        pass


def test_node_locality_mismatch_is_rejected():
    # 4 ranks laid out 2 per node (local ranks 0,1,0,1) but all claiming one host: the hostname
    # all-gather sees local ranks [0, 0, 1, 1] there and rejects the layout
    with pytest.raises(AssertionError, match="TopologyError"):
        run_ranks(_bad_topology_rank, 4, env={"DDL_HOSTNAME": "same-host"}, nodes=2)


def test_explicit_backend_builds_a_one_rank_group():
    """DDL_BACKEND at world size 1 builds a 1-rank group, so the exchange path runs (and can be
    timed) on a single device; without it a lone rank has no group and no exchange."""
    res, = run_ranks(_exchange_rank, 1, "alltoall", 0.5, env={"DDL_BACKEND": "gloo"})
    eps, n_ex = res
    assert n_ex == 20
    for rows in eps:  # world 1: every exchanged row comes back to its own window
        assert len({tuple(x) for x in rows[:, :3].tolist()}) == len(rows) == 40


def test_init_mpi_error_handling_rejects_non_multiple():
    from ddl_amd.exceptions import TopologyError
    from ddl_amd.parallel import init_mpi_error_handling
    from ddl_amd.types import DDLEnv

    init_mpi_error_handling(DDLEnv(rank=0, world_size=8), 4)
    init_mpi_error_handling(DDLEnv(rank=0, world_size=1), 1)  # single rank: warning only
    with pytest.raises(TopologyError):
        init_mpi_error_handling(DDLEnv(rank=0, world_size=6), 4)


def _indexed_zero_copy_rank(rank, world, name, n, gb, epochs):
    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.zerocopy import ZeroCopyLoader

    src = SharedArraySource(name, n, (2,), "int64")
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ZeroCopyLoader(src, gb, env, seed=5, n_epochs=epochs, device="cpu")
        return [[b[:, 0].clone().numpy() for b in dl] for _ in range(epochs)]


def test_indexed_headline_order_is_world_size_invariant():
    """bench.py's ``indexed`` order (ZeroCopyLoader over a node-shared source): the union of the ranks'
    slices of every global batch -- in rank order -- is the same batch at W = 1, 2, 4 and 8."""
    import numpy as np

    from ddl_amd.models import SharedArraySource

    n, gb, epochs = 500, 64, 2
    data = torch.stack([torch.arange(n), torch.arange(n) * 3], 1).to(torch.int64)
    src = SharedArraySource.create(f"ddl_amd_inv_{np.random.randint(1 << 30)}", data)
    try:
        merged = {}
        for world in (1, 2, 4, 8):
            res = run_ranks(_indexed_zero_copy_rank, world, src.name, n, gb, epochs)
            merged[world] = [[np.concatenate([res[r][e][g] for r in range(world)]) for g in range(len(res[0][e]))]
                             for e in range(epochs)]
        for world in (2, 4, 8):
            for e in range(epochs):
                assert len(merged[world][e]) == len(merged[1][e]) == n // gb
                for a, b in zip(merged[world][e], merged[1][e]):
                    assert np.array_equal(a, b)
        assert not np.array_equal(np.concatenate(merged[1][0]), np.concatenate(merged[1][1]))  # fresh order per epoch
    finally:
        src.close()


def _token_rank(rank, world, name, n, max_len, gb, k, resume=None, stop_after=None):
    """Pad-mode token loader with k-batch windows: each rank's batches as lists of sequence ids
    (the first token of every synthetic sequence is checked against the corpus instead)."""
    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer

    offs = SharedArraySource(name + "_off", n + 1, (1,), "int64")
    n_tok = int(offs.tensor()[-1])
    src = SharedTokenSource(SharedArraySource(name + "_tok", n_tok, (1,), "int32"), offs, max_len)
    starts = offs.tensor().view(-1).numpy()
    toks = src.tokens.tensor().view(-1).numpy()
    out = []
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(TokenBatchProducer(src, gb, max_len, "pad", batches_per_window=k),
                                           gb // world, conn, 1, env=env, auto_mark=True, resume_state=resume,
                                           output=ddl_amd.OutputSpec(collate="tokens"),
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=5))
        for i, b in enumerate(dl):
            ids = b["input_ids"]
            # identify each row's sequence by its tokens (synthetic corpus: rows are distinct)
            seqs = []
            for r in range(ids.shape[0]):
                n_r = int(b["attention_mask"][r].sum())
                hit = [j for j in range(n) if starts[j + 1] - starts[j] == n_r
                       and np.array_equal(toks[starts[j]:starts[j + 1]], ids[r, :n_r].numpy())]
                seqs.append(hit[0] if len(hit) == 1 else -1)
            out.append(seqs)
            if stop_after is not None and i + 1 == stop_after:
                sd = dl.state_dict()
                dl.close()
                return out, sd
    return out, None


@pytest.fixture
def token_corpus():
    from ddl_amd.models.tokens import SharedTokenSource

    src = SharedTokenSource.synthetic(f"ddl_amd_mrtok_{np.random.randint(1 << 30)}", 96, 4, 64, seed=2)
    yield src
    src.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_token_windows_world_size_invariant(token_corpus, world):
    """k-batch token windows keep the indexed order: global batch g = concat of rank slices, at any W."""
    from ddl_amd.permutation import EpochOrder

    src, gb, k = token_corpus, 8, 4
    res = run_ranks(_token_rank, world, src.tokens.name[:-4], src.n, src.max_len, gb, k, env={"DDL_DEVICE": "cpu"})
    order = EpochOrder(src.n, gb, 5)
    for g in range(order.batches_per_epoch):
        merged = sum((r[0][g] for r in res), [])
        assert merged == [int(x) for x in order.indices(0, g)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("save_world,resume_world", [(2, 1), (4, 8), (8, 2)])
def test_token_windows_resume_mid_window_at_other_world_size(token_corpus, save_world, resume_world):
    """Checkpoint a k-batch token loader mid-window (global batch 6 = window 1, sub-batch 2) at one world
    size and resume at another: the resumed ranks' slices merge into exactly the remaining global batches."""
    from ddl_amd.permutation import EpochOrder

    src, gb, k = token_corpus, 8, 4
    res = run_ranks(_token_rank, save_world, src.tokens.name[:-4], src.n, src.max_len, gb, k, None, 6,
                    env={"DDL_DEVICE": "cpu"})
    sd = res[0][1]
    assert all(r[1]["global_batch_cursor"] == 6 for r in res) and sd["batches_per_window"] == k
    out = run_ranks(_token_rank, resume_world, src.tokens.name[:-4], src.n, src.max_len, gb, k, sd,
                    env={"DDL_DEVICE": "cpu"})
    order = EpochOrder(src.n, gb, 5)
    merged = [sum((r[0][i] for r in out), []) for i in range(len(out[0][0]))]
    assert merged == [[int(x) for x in order.indices(0, g)] for g in range(6, order.batches_per_epoch)]
