"""Map-style Dataset drop-in: ``IndexedProducer(MapDatasetSource(ds))`` delivers batches in the
dataset's own sample structure, in the world-size-invariant global order."""

import os

import numpy as np
import pytest
import torch

import ddl_amd
from ddl_amd.exceptions import ShapeMismatchError
from ddl_amd.models import IndexedProducer, MapDatasetSource, unpack_fields
from ddl_amd.permutation import EpochOrder
from tests.mp_harness import run_ranks


class TupleDataset(torch.utils.data.Dataset):
    """image uint8 [3, 5, 7], label int, weight float32, bf16 feature [4], flag bool."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(i)
        img = torch.randint(0, 256, (3, 5, 7), generator=g, dtype=torch.uint8)
        return (img, i * 7, np.float32(i) / 3, torch.full((4,), float(i), dtype=torch.bfloat16), bool(i % 2))


class DictDataset(TupleDataset):
    def __getitem__(self, i):
        img, label, w, feat, flag = super().__getitem__(i)
        return {"image": img, "label": label, "weight": w}


def _expected(ds, idx):
    return torch.utils.data.default_collate([ds[int(i)] for i in idx])


def _check(batch, ref):
    if isinstance(ref, dict):
        assert set(batch) == set(ref)
        pairs = [(batch[k], ref[k]) for k in ref]
    else:
        pairs = list(zip(batch, ref))
    for got, want in pairs:
        want = torch.as_tensor(want)
        assert got.shape == want.shape and got.dtype == want.dtype, (got.shape, want.shape, got.dtype, want.dtype)
        assert torch.equal(got.cpu(), want)


def test_layout_and_unpack_roundtrip():
    ds = TupleDataset(10)
    src = MapDatasetSource(ds)
    assert src.kind == "tuple" and len(src.fields) == 5
    assert all(off % 16 == 0 for _, _, _, off, _ in src.fields) and src.row_bytes % 16 == 0
    rows = np.zeros((4, src.row_bytes), dtype=np.uint8)
    src.gather(np.array([3, 1, 4, 1]), rows.ctypes.data, n_threads=1)
    _check(unpack_fields(torch.from_numpy(rows), src.fields, src.kind), _expected(ds, [3, 1, 4, 1]))


class ViewDataset(torch.utils.data.Dataset):
    """Fields that are views: a row of a shared table (storage offset), a transposed (non-contiguous)
    tensor and a strided numpy slice -- the native span copy must see their real bytes."""

    def __init__(self, n):
        self.n = n
        self.table = torch.arange(n * 3 * 8 * 8, dtype=torch.int16).view(n, 3, 8, 8)
        self.np_table = np.arange(n * 12, dtype=np.float32).reshape(n, 12)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return self.table[i], self.table[i].transpose(1, 2), self.np_table[i, ::2], i


@pytest.mark.parametrize("n_threads", [1, 4])
def test_views_and_threaded_span_copy(n_threads):
    ds = ViewDataset(300)
    src = MapDatasetSource(ds)
    idx = np.random.default_rng(0).permutation(300)[:200]
    rows = np.zeros((len(idx), src.row_bytes), dtype=np.uint8)
    src.gather(idx, rows.ctypes.data, n_threads=n_threads)
    _check(unpack_fields(torch.from_numpy(rows), src.fields, src.kind), _expected(ds, idx))


def test_inconsistent_sample_is_rejected():
    class Bad(TupleDataset):
        def __getitem__(self, i):
            out = super().__getitem__(i)
            return out if i == 0 else out[:4]

    src = MapDatasetSource(Bad(4))
    rows = np.zeros((2, src.row_bytes), dtype=np.uint8)
    with pytest.raises(ValueError, match="fields"):
        src.gather(np.array([0, 1]), rows.ctypes.data, n_threads=1)


@pytest.mark.parametrize("ds_cls", [TupleDataset, DictDataset])
def test_map_dataset_loader_cpu(ds_cls, monkeypatch):
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    ds, gb = ds_cls(50), 8
    order = EpochOrder(len(ds), gb, 3)
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(MapDatasetSource(ds), gb, host_threads=2), gb, conn, 2,
                                           env=env, auto_mark=True, order=ddl_amd.OrderSpec(mode="indexed", seed=3))
        for e in range(2):
            n = 0
            for g, b in enumerate(dl):
                _check(b, _expected(ds, order.indices(e, g)))
                n += 1
            assert n == order.batches_per_epoch


def _rank(rank, world, n, gb):
    import ddl_amd

    out = []
    ds = TupleDataset(n)
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(MapDatasetSource(ds), gb), gb // world, conn, 1, env=env,
                                           auto_mark=True, order=ddl_amd.OrderSpec(mode="indexed", seed=3))
        for b in dl:
            out.append(b[1].tolist())  # labels = 7 * sample id
    return out


@pytest.mark.parametrize("world", [1, 2])
def test_map_dataset_world_size_invariant(world):
    n, gb = 40, 8
    res = run_ranks(_rank, world, n, gb, env={"DDL_DEVICE": "cpu"})
    order = EpochOrder(n, gb, 3)
    for g in range(order.batches_per_epoch):
        merged = sum((r[g] for r in res), [])
        assert merged == [7 * int(i) for i in order.indices(0, g)]


@pytest.mark.gpu
@pytest.mark.parametrize("native", [True, False])
def test_map_dataset_loader_gpu(native):
    ds, gb = TupleDataset(64), 16
    order = EpochOrder(len(ds), gb, 3)
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(MapDatasetSource(ds), gb), gb, conn, 2, env=env,
                                           auto_mark=True, staging=ddl_amd.StagingSpec(native_dispatch=native),
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=3))
        for e in range(2):
            for g, b in enumerate(dl):
                assert all(t.is_cuda for t in b)
                _check(b, _expected(ds, order.indices(e, g)))
        st = dl.stats()
    assert (st.get("native_dispatch") is not None) == native


def test_dataloader_front_end_cpu(monkeypatch):
    """``ddl_amd.DataLoader(dataset, batch_size, shuffle=...)``: torch DataLoader surface over the
    indexed loader -- epochs via repeated iter(), len, shuffle=False order, state_dict round trip."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    ds, bs = TupleDataset(40), 8
    order = EpochOrder(len(ds), bs, 5)
    with ddl_amd.DataLoader(ds, batch_size=bs, shuffle=True, num_workers=2, seed=5) as dl:
        assert len(dl) == order.batches_per_epoch
        for e in range(2):
            got = [b[1].tolist() for b in dl]
            assert got == [[7 * int(i) for i in order.indices(e, g)] for g in range(order.batches_per_epoch)]
        it = iter(dl)
        next(it)
        next(it)
        sd = dl.state_dict()
        assert sd["epoch"] == 2 and sd["global_batch_cursor"] == 2
    with ddl_amd.DataLoader(ds, batch_size=bs, shuffle=True, num_workers=2, seed=5, resume_state=sd) as dl:
        rest = [b[1].tolist() for b in dl]
        assert rest == [[7 * int(i) for i in order.indices(2, g)] for g in range(2, order.batches_per_epoch)]
    with ddl_amd.DataLoader(ds, batch_size=bs, shuffle=False, drop_last=True, num_workers=1) as dl:
        labels = [x for b in dl for x in b[1].tolist()]
        assert labels == [7 * i for i in range(len(ds))]
    # drop_last=False: the last batch is completed from the start of the epoch (DistributedSampler-style)
    with ddl_amd.DataLoader(TupleDataset(43), batch_size=bs, shuffle=False, drop_last=False, num_workers=2) as dl:
        labels = [x for b in dl for x in b[1].tolist()]
        assert labels == [7 * (i % 43) for i in range(48)]
        it = iter(dl)
        next(it)
        sd43 = dl.state_dict()
    assert sd43["drop_last"] is False
    # a checkpoint taken with one drop_last does not resume under the other: the error names the cause
    with pytest.raises(ShapeMismatchError, match="drop_last"):
        ddl_amd.DataLoader(TupleDataset(43), batch_size=bs, shuffle=False, drop_last=True, num_workers=1,
                           resume_state=sd43)


def _train_and_eval_rank(rank, world, bs):
    """A training loader and an evaluation loader alive together (the usual torch program): one launcher
    session; closing the training loader keeps the process group (a DDP model's) and the eval loader working."""
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd import frontend

    train, val = TupleDataset(48), DictDataset(40)
    tl = ddl_amd.DataLoader(train, batch_size=bs, shuffle=True, num_workers=2, seed=1)
    vl = ddl_amd.DataLoader(val, batch_size=bs, shuffle=False, drop_last=True, num_workers=1)
    assert frontend._Session.current.refs == 2 and tl.env is vl.env
    got_train = [b[1].tolist() for b in tl]
    tl.close()
    assert dist.is_initialized()  # the eval loader's session keeps the group
    t = torch.ones(1)
    dist.all_reduce(t)
    got_val = [b["label"].tolist() for b in vl]
    vl.close()
    assert frontend._Session.current is None and not dist.is_initialized()
    return got_train, got_val, float(t)


def test_dataloader_front_end_train_and_eval():
    bs, world = 4, 2
    res = run_ranks(_train_and_eval_rank, world, bs, env={"DDL_DEVICE": "cpu"})
    tr, va = EpochOrder(48, bs * world, 1), EpochOrder(40, bs * world, 0, shuffle=False)
    for r, (got_train, got_val, total) in enumerate(res):
        assert total == world
        assert got_train == [[7 * int(i) for i in tr.indices(0, g)[r * bs:(r + 1) * bs]]
                             for g in range(tr.batches_per_epoch)]
        assert got_val == [[7 * int(i) for i in va.indices(0, g)[r * bs:(r + 1) * bs]]
                           for g in range(va.batches_per_epoch)]


def _mark_worker(path, worker_id):
    open(os.path.join(path, f"worker{worker_id}"), "w").close()


def test_dataloader_front_end_torch_arguments(monkeypatch, tmp_path):
    """torch's DataLoader signature: positional (dataset, batch_size, shuffle), num_workers=0 (one in-process
    worker thread), worker_init_fn in every worker, generator as the seed, the no-op pinning / persistence
    arguments; sampler / collate_fn / iterable datasets are refused with the reason."""
    import functools
    import threading

    monkeypatch.setenv("DDL_DEVICE", "cpu")
    ds, bs = TupleDataset(24), 4
    g = torch.Generator().manual_seed(11)
    kw = dict(pin_memory=True, persistent_workers=True, prefetch_factor=2, multiprocessing_context="spawn",
              timeout=30)
    with ddl_amd.DataLoader(ds, bs, True, num_workers=0, generator=g, **kw) as dl:
        assert all(isinstance(p, threading.Thread) for p in dl._conn.processes)
        got = [b[1].tolist() for b in dl]
    order = EpochOrder(len(ds), bs, 11)
    assert got == [[7 * int(i) for i in order.indices(0, k)] for k in range(order.batches_per_epoch)]
    with ddl_amd.DataLoader(ds, batch_size=bs, num_workers=2, collate_fn=torch.utils.data.default_collate,
                            worker_init_fn=functools.partial(_mark_worker, str(tmp_path))) as dl:
        assert [x for b in dl for x in b[1].tolist()] == [7 * i for i in range(len(ds))]  # shuffle defaults off
    assert sorted(os.listdir(tmp_path)) == ["worker0", "worker1"]
    with pytest.raises(ValueError, match="sampler"):
        ddl_amd.DataLoader(ds, batch_size=bs, sampler=torch.utils.data.SequentialSampler(ds))
    with pytest.raises(ValueError, match="collate_fn"):
        ddl_amd.DataLoader(ds, batch_size=bs, collate_fn=lambda b: b)

    class Stream(torch.utils.data.IterableDataset):
        def __iter__(self):
            return iter(range(3))

    with pytest.raises(TypeError, match="map-style"):
        ddl_amd.DataLoader(Stream(), batch_size=bs)
    from ddl_amd import frontend

    assert frontend._Session.current is None  # refused loaders leave no session behind


@pytest.mark.gpu
def test_dataloader_front_end_gpu():
    ds, bs = TupleDataset(64), 16
    order = EpochOrder(len(ds), bs, 5)
    with ddl_amd.DataLoader(ds, batch_size=bs, shuffle=True, num_workers=2, seed=5) as dl:
        for e in range(2):
            for g, b in enumerate(dl):
                assert b[0].is_cuda and b[0].shape == (bs, 3, 5, 7)
                _check(b, _expected(ds, order.indices(e, g)))


@pytest.mark.gpu
def test_dataloader_front_end_train_and_eval_gpu():
    """A training loader in use on the GPU, then an evaluation loader created mid-run (its workers spawned
    after the GPU is initialised) and interleaved with it; closing the training loader first."""
    ds, val, bs = TupleDataset(64), DictDataset(80), 16
    order, vorder = EpochOrder(len(ds), bs, 5), EpochOrder(len(val), bs, 0, shuffle=False)
    tl = ddl_amd.DataLoader(ds, batch_size=bs, shuffle=True, num_workers=2, seed=5)
    it = iter(tl)
    _check(next(it), _expected(ds, order.indices(0, 0)))
    vl = ddl_amd.DataLoader(val, batch_size=bs, num_workers=0)  # shuffle off (eval), an in-process worker
    vit = iter(vl)
    for g in range(1, order.batches_per_epoch):
        _check(next(it), _expected(ds, order.indices(0, g)))
        _check(next(vit), _expected(val, vorder.indices(0, g - 1)))
    tl.close()
    b = next(vit)
    assert b["image"].is_cuda
    _check(b, _expected(val, vorder.indices(0, order.batches_per_epoch - 1)))
    vl.close()
