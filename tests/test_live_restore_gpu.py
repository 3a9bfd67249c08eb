"""Live restore on the DEVICE path for every loader family (reference cursor: epoch / batch /
target_rank, reference ddl/mpi_dataloader.py:119-121).

``load_state_dict`` mid-window and a repositioning ``set_epoch`` drain the staging ring, move the
producers and rebuild the stager + native engine. Each test compares the batches delivered after the
restore bit for bit with an uninterrupted run of the same loader, for

* token windows (k sub-batches per window, pad and pack) in native inline, whole-window and Python
  dispatch -- the stager's per-window meta table must survive the rebuild;
* a uint8 -> bf16 normalised image loader with the per-window device shuffle.

The exchange-on loader (1-rank RCCL group) is covered in ``test_exchange_gpu.py``.
"""

import numpy as np
import pytest
import torch

import ddl_amd
from ddl_amd import Marker
from ddl_amd.models.producers import ImageWindowProducer
from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer

pytestmark = pytest.mark.gpu


def _host(b):
    if isinstance(b, dict):
        return {k: (v.cpu().clone() if isinstance(v, torch.Tensor) else v) for k, v in b.items()}
    return tuple(t.cpu().clone() for t in b)


def _same(a, b):
    if isinstance(a, dict):
        assert a.keys() == b.keys()
        for k in a:
            if isinstance(a[k], torch.Tensor):
                assert a[k].dtype == b[k].dtype and torch.equal(a[k], b[k]), k
            else:
                assert a[k] == b[k], k
        return
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype and torch.equal(x, y)


def _take(dl, n):
    """Up to n batches with the reference's mark loop (END_OF_EPOCH at each epoch end)."""
    out = []
    while len(out) < n and dl.epoch < dl.n_epochs:
        for i in range(dl.epoch_batch, len(dl)):
            out.append(_host(dl[i]))
            dl.mark(Marker.END_OF_BATCH)
            if len(out) == n:
                if dl.epoch_batch == len(dl):
                    dl.mark(Marker.END_OF_EPOCH)
                return out
        dl.mark(Marker.END_OF_EPOCH)
    return out


@pytest.fixture(scope="module")
def corpus():
    src = SharedTokenSource.synthetic(f"ddl_amd_live_{np.random.randint(1 << 30)}", 200, 5, 300, seed=3)
    yield src
    src.close()


def _token_loader(corpus, conn, env, mode, dispatch, epochs=2):
    return ddl_amd.DistributedDataLoader(TokenBatchProducer(corpus, 16, 256, mode, batches_per_window=4), 16, conn,
                                         epochs, env=env, output=ddl_amd.OutputSpec(collate="tokens"),
                                         staging=ddl_amd.StagingSpec(native_dispatch=dispatch),
                                         order=ddl_amd.OrderSpec(mode="indexed", seed=4))


@pytest.mark.parametrize("dispatch", ["inline", "window", False])
@pytest.mark.parametrize("mode", ["pad", "pack"])
def test_token_loader_live_load_state_dict(corpus, mode, dispatch):
    """Checkpoint mid-window (global batch 6 = window 1, sub-batch 2), run 3 more, restore: the rest
    equals the uninterrupted run (the stager rebuilt by the seek keeps the token meta table)."""
    with ddl_amd.start(n_producers=2) as (env, conn):
        full = _take(_token_loader(corpus, conn, env, mode, dispatch), 10 ** 9)
    assert len(full) == 24
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = _token_loader(corpus, conn, env, mode, dispatch)
        assert dl.device.type == "cuda" and dl._stager.meta_bytes > 0
        head = _take(dl, 6)
        sd = dl.state_dict()
        _take(dl, 3)
        dl.load_state_dict(sd)
        assert dl._stager.meta_bytes > 0
        if dispatch:
            assert dl._engine is not None and dl.stats()["native_dispatch"]["mode"] == dispatch
        tail = _take(dl, 10 ** 9)
    assert len(head) + len(tail) == len(full)
    for a, b in zip(head + tail, full):
        _same(a, b)
        assert a["n_tokens"] > 0


@pytest.mark.parametrize("dispatch", ["window", False])
def test_token_loader_live_set_epoch(corpus, dispatch):
    """A repositioning set_epoch mid-epoch (jump to epoch 1, then back to 0) on the device path."""
    with ddl_amd.start(n_producers=2) as (env, conn):
        full = _take(_token_loader(corpus, conn, env, "pack", dispatch), 10 ** 9)
    per_epoch = len(full) // 2
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = _token_loader(corpus, conn, env, "pack", dispatch)
        _take(dl, 5)
        dl.set_epoch(1)
        e1 = _take(dl, per_epoch)
        assert len(e1) == per_epoch
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = _token_loader(corpus, conn, env, "pack", dispatch)
        _take(dl, 7)
        dl.set_epoch(0)  # restart the current epoch
        e0 = _take(dl, per_epoch)
    for a, b in zip(e1, full[per_epoch:]):
        _same(a, b)
    for a, b in zip(e0, full[:per_epoch]):
        _same(a, b)


def _image_loader(conn, env, dispatch, epochs=3):
    norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225]}
    return ddl_amd.DistributedDataLoader(ImageWindowProducer(16, (3, 8, 8), "uint8", seed=5), 4, conn, epochs, env=env,
                                         output=ddl_amd.OutputSpec(dtype=torch.bfloat16, normalize=norm),
                                         staging=ddl_amd.StagingSpec(native_dispatch=dispatch),
                                         order=ddl_amd.OrderSpec(shuffle="device", seed=9))


@pytest.mark.parametrize("dispatch", ["auto", "lookahead", False])
def test_normalised_image_loader_live_restore(dispatch):
    """uint8 windows -> fused gather + normalise -> bf16, with the per-window device shuffle: a live
    load_state_dict mid-window and a set_epoch rewind both continue exactly as the full run."""
    with ddl_amd.start(n_producers=3) as (env, conn):
        full = _take(_image_loader(conn, env, dispatch), 10 ** 9)
    assert len(full) == 12 and full[0][0].dtype == torch.bfloat16
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = _image_loader(conn, env, dispatch)
        head = _take(dl, 5)
        sd = dl.state_dict()
        _take(dl, 4)
        dl.load_state_dict(sd)
        tail = _take(dl, 3)
        dl.set_epoch(1)
        e1 = _take(dl, 4)
    for a, b in zip(head + tail, full):
        _same(a, b)
    for a, b in zip(e1, full[4:8]):
        _same(a, b)
