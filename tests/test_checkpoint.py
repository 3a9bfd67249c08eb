"""Drop-in checkpointing: live ``load_state_dict``, ``set_epoch``, resume with a different slot count.

The reference has no checkpoint at all; its implicit cursor is ``epoch / batch / target_rank``
(reference ddl/mpi_dataloader.py:119-121). Here the cursor is restored on a LIVE loader: the
producers are repositioned in place (``Connection.seek_producers``) and the staging ring is rebuilt,
and every test compares the delivered batches bit for bit against an uninterrupted run.
"""

import pytest
import torch

import ddl_amd
from ddl_amd import Marker
from ddl_amd.exceptions import ShapeMismatchError
from tests.helpers import IdProducer

EPOCHS = 3
KW = dict(output=ddl_amd.OutputSpec(copy_batches=True), order=ddl_amd.OrderSpec(shuffle="device", seed=7))


def _device():
    return "cuda" if torch.cuda.is_available() else "cpu"


@pytest.fixture(autouse=True)
def _host_path(monkeypatch, request):
    if "gpu" not in request.keywords:
        monkeypatch.setenv("DDL_DEVICE", "cpu")


def _take(dl, n):
    """Consume up to n batches (marking as the reference loop does); returns the rows."""
    out = []
    while len(out) < n and dl.epoch < dl.n_epochs:
        for i in range(dl.epoch_batch, len(dl)):
            out.append(torch.cat([b.reshape(b.shape[0], -1) for b in dl[i]], 1).cpu().clone())
            dl.mark(Marker.END_OF_BATCH)
            if len(out) == n:
                if dl.epoch_batch == len(dl):
                    dl.mark(Marker.END_OF_EPOCH)
                return out
        dl.mark(Marker.END_OF_EPOCH)
    return out


def _full(n_slots=1, n_producers=3):
    with ddl_amd.start(n_producers=n_producers) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW,
                                           staging=ddl_amd.StagingSpec(n_slots=n_slots))
        return _take(dl, 10 ** 9)


@pytest.mark.parametrize("at", [2, 6, 9])
def test_load_state_dict_on_live_loader(at):
    """Checkpoint after `at` batches, run on 3 more, then load_state_dict: the rest equals the
    uninterrupted run from the checkpoint on (window boundary, mid-window, across epochs)."""
    full = _full()
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW)
        head = _take(dl, at)
        sd = dl.state_dict()
        _take(dl, min(3, 11 - at))  # moves on (past a window / epoch boundary), not to the end of the run
        dl.load_state_dict(sd)
        tail = _take(dl, 10 ** 9)
    assert len(head) + len(tail) == len(full) == 12
    for a, b in zip(head + tail, full):
        assert torch.equal(a, b)


def test_load_state_dict_rewinds_and_fast_forwards():
    full = _full()
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW)
        _take(dl, 1)
        sd1 = dl.state_dict()
        _take(dl, 7)
        sd8 = dl.state_dict()
        dl.load_state_dict(sd1)  # back
        again = _take(dl, 2)
        dl.load_state_dict(sd8)  # forward again
        rest = _take(dl, 10 ** 9)
    assert all(torch.equal(a, b) for a, b in zip(again, full[1:3]))
    assert len(rest) == 4 and all(torch.equal(a, b) for a, b in zip(rest, full[8:]))


def test_set_epoch_positions_at_epoch_start():
    full = _full()
    per_epoch = len(full) // EPOCHS
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW)
        dl.set_epoch(0)  # already there: no-op
        _take(dl, 1)
        dl.set_epoch(2)  # jump ahead mid-epoch
        e2 = _take(dl, per_epoch)
        assert dl.epoch == EPOCHS or dl._finalized
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW)
        _take(dl, per_epoch + 2)
        dl.set_epoch(1)  # restart the current epoch
        e1 = _take(dl, per_epoch)
        dl.set_epoch(0)  # and go back
        e0 = _take(dl, per_epoch)
    assert all(torch.equal(a, b) for a, b in zip(e2, full[2 * per_epoch:]))
    assert all(torch.equal(a, b) for a, b in zip(e1, full[per_epoch:2 * per_epoch]))
    assert all(torch.equal(a, b) for a, b in zip(e0, full[:per_epoch]))


def test_resume_with_a_different_slot_count():
    """Window content is a function of (producer, round), not of the slot: n_slots may change."""
    full = _full(n_slots=1)
    assert all(torch.equal(a, b) for a, b in zip(_full(n_slots=2), full))
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW,
                                           staging=ddl_amd.StagingSpec(n_slots=1))
        head = _take(dl, 5)
        sd = dl.state_dict()
        dl.close()
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, resume_state=sd, **KW,
                                           staging=ddl_amd.StagingSpec(n_slots=3))
        tail = _take(dl, 10 ** 9)
    assert all(torch.equal(a, b) for a, b in zip(head + tail, full))


def test_window_checkpoint_rejects_other_producer_count():
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW)
        _take(dl, 2)
        sd = dl.state_dict()
        dl.close()
    with ddl_amd.start(n_producers=2) as (env, conn):
        with pytest.raises(ShapeMismatchError, match="producers"):
            ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, resume_state=sd, **KW)


def test_perm_key_distinct_beyond_256_producers():
    """The device-permutation key of a window visit mixes (producer, round) into 64 bits: no aliasing
    between producer p and p + 256 (the old (round << 8) | p key aliased them)."""
    from ddl_amd.dataloader import window_perm_key

    keys = {window_perm_key(p, r) for p in range(600) for r in range(40)}
    assert len(keys) == 600 * 40
    assert all(0 <= k < (1 << 63) for k in keys)


@pytest.mark.gpu
def test_load_state_dict_live_on_gpu():
    """Device path: staged HBM ring drained and rebuilt; the resumed batches equal the uninterrupted run."""
    full = _full()
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, EPOCHS, env=env, **KW)
        assert dl.device.type == "cuda"
        head = _take(dl, 6)
        sd = dl.state_dict()
        _take(dl, 4)
        dl.load_state_dict(sd)
        tail = _take(dl, 10 ** 9)
    assert all(torch.equal(a, b) for a, b in zip(head + tail, full))


def test_sample_index_cursor_in_indexed_checkpoints():
    """Indexed checkpoints carry the epoch/sample-index position too; a state with only
    ``global_sample_cursor`` resumes at the same global batch."""
    from ddl_amd.permutation import batch_cursor

    sd = {"global_batch_cursor": 5, "global_sample_cursor": 5 * 64}
    assert batch_cursor(sd, 64) == 5
    assert batch_cursor({"global_sample_cursor": 320}, 64) == 5
    with pytest.raises(ValueError):
        batch_cursor({"global_sample_cursor": 321}, 64)
