"""Consumer/producer engine on CPU with real producer processes (SURVEY §4.4 level 2).

Replaces the reference's only test (``mpirun -np 4 python3 run_ddl.py``,
reference tests/test_ddl.py:8-28, which checks no data) with assertions on
shapes, window round-robin, exactly-once delivery, determinism, resume and
failure handling.
"""

import numpy as np
import pytest
import torch

import ddl_amd
from ddl_amd import Marker
from ddl_amd.exceptions import DDLTimeoutError, PeerDeathError, ShapeMismatchError
from ddl_amd.models import PointwiseProducer
from tests.helpers import FailingProducer, IdProducer


@pytest.fixture(autouse=True)
def _host_path(monkeypatch):
    """These tests cover the host (CPU) data path even on a GPU box; the device path is test_loader_gpu.py."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")


def _epochs(dl, n_epochs, collect=True):
    out = []
    for _ in range(n_epochs):
        rows = []
        for i, batch in enumerate(dl):
            if collect:
                rows.append(torch.cat([b.reshape(b.shape[0], -1) for b in batch], 1).clone())
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)
        out.append(torch.cat(rows) if rows else None)
    return out


def test_reference_harness_config_parity():
    """BASELINE config 1 layout: 1 consumer + 3 producers, nData=10 timesteps, batch 4096, splits (3,5,1)."""
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(PointwiseProducer(n_timesteps=10), 4096, conn, 3, 0.5,
                                           "sendrecv_replace", 0, 1, env=env)
        assert dl.device.type == "cpu"
        assert len(dl) == 24  # 100,520 // 4096
        windows = []
        for epoch in range(3):
            n = 0
            for i, (pos, target, w) in enumerate(dl):
                assert pos.shape == (4096, 3) and target.shape == (4096, 5) and w.shape == (4096, 1)
                assert pos.dtype == torch.float32
                n += 1
                dl.mark(Marker.END_OF_BATCH)
            windows.append(dl.target_rank)
            assert n == 24
            dl.mark(Marker.END_OF_EPOCH)
        assert dl._finalized


def test_round_robin_windows_and_exactly_once():
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(48, 6), 8, conn, 7, env=env)
        eps = _epochs(dl, 7)
    for e, rows in enumerate(eps):
        assert rows.shape == (48, 6)
        assert rows[:, 1].unique().tolist() == [e % 3]          # window order 1,2,3,1,2,3,1 (reference §3.4)
        assert rows[:, 3].unique().tolist() == [e // 3]         # producer round
        assert rows[:, 2].tolist() == list(range(48))           # exactly once, window order
        assert torch.equal(rows[:, 4], rows[:, 2] * 7 + 4)


def test_zero_copy_views_alias_the_window():
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 1, env=env)
        a, b = dl[0]
        _, win = dl.arys[0][0]
        assert a.data_ptr() == win.data_ptr()  # reference semantics: views of the shared window
        for i in range(len(dl)):
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)


def test_split_along_epoch_mode():
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(32, 4), 8, conn, 2, env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           order=ddl_amd.OrderSpec(mode="split_along_epoch"))
        assert len(dl) == 12
        eps = _epochs(dl, 2)
    for e, rows in enumerate(eps):
        assert rows.shape == (96, 4)
        assert rows[:, 1].tolist() == [0] * 32 + [1] * 32 + [2] * 32
        assert rows[:, 3].unique().tolist() == [e]


def test_auto_mark_dataloader_dropin_with_slots():
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(20, 4), 5, conn, 4, env=env, auto_mark=True,
                                           staging=ddl_amd.StagingSpec(n_slots=2))
        seen = []
        for epoch in range(4):
            seen.append(torch.cat([torch.cat(b, 1) for b in dl]))
    for e, rows in enumerate(seen):
        assert rows[:, 2].tolist() == list(range(20))
        assert rows[:, 1].unique().tolist() == [e % 2]


@pytest.mark.parametrize("auto_mark", [False, True])
def test_column_normalisation_applies_with_owned_batches(auto_mark):
    # per-column affine on tabular windows; owned (contiguous) batches must not skip it
    mean, std = [1.0, 2.0, 3.0, 4.0], [2.0, 4.0, 0.5, 1.0]
    with ddl_amd.start(n_producers=1) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(20, 4, dtype="float32"), 5, conn, 1, env=env,
                                           auto_mark=auto_mark,
                                           output=ddl_amd.OutputSpec(normalize={"mean": mean, "std": std}))
        got = []
        for b in dl:
            assert all(t.is_contiguous() for t in b) or not auto_mark
            got.append(torch.cat(b, 1).clone())
            if not auto_mark:
                dl.mark(Marker.END_OF_BATCH)
        if not auto_mark:
            dl.mark(Marker.END_OF_EPOCH)
    rows = torch.cat(got)
    i = torch.arange(20, dtype=torch.float32)
    raw = torch.stack([torch.zeros(20), torch.zeros(20), i, torch.zeros(20)], 1)
    ref = (raw - torch.tensor(mean)) / torch.tensor(std)
    torch.testing.assert_close(rows, ref)


def test_host_device_shuffle_uses_feistel_order():
    from ddl_amd.dataloader import window_perm_key
    from ddl_amd.permutation import FeistelPermutation

    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(40, 4), 8, conn, 2, env=env,
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=3))
        eps = _epochs(dl, 2)
    for e, rows in enumerate(eps):
        perm = FeistelPermutation(40, 3, window_perm_key(e, 0)).full()  # window e: producer e, round 0
        assert np.array_equal(rows[:, 2].numpy(), perm)


def test_single_rank_without_producers_has_len_zero():
    with ddl_amd.start(n_producers=0) as (env, conn):
        assert conn is None
        dl = ddl_amd.DistributedDataLoader(IdProducer(), 4, conn, 2)
        assert len(dl) == 0
        assert list(dl) == []


def test_decorator_forwards_kwargs_and_runs_producers():
    @ddl_amd.distributed_dataloader(n_producers=2)
    def main(cfg, env, conn, *, extra=None):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), cfg, conn, 2, env=env)
        n = sum(1 for _ in _epochs(dl, 2, collect=False))
        return env.n_producers, extra, n

    assert main(4, extra="kw") == (2, "kw", 2)  # reference drops kwargs (ddl/ddl_env.py:116)


def test_thread_mode_producers(monkeypatch):
    monkeypatch.setenv("DDL_PRODUCER_MODE", "thread")
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 3, env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True))
        eps = _epochs(dl, 3)
    assert [r[:, 1].unique().item() for r in eps] == [0, 1, 0]


def test_resume_from_state_dict():
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 5, env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True))
        first = _epochs(dl, 2)
        sd = dl.state_dict()
        dl.close()
    assert sd["epoch"] == 2 and sd["window"] == 2 and sd["batch"] == 0
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 5, env=env, resume_state=sd,
                                           output=ddl_amd.OutputSpec(copy_batches=True))
        rest = _epochs(dl, 3)
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 5, env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True))
        full = _epochs(dl, 5)
    for a, b in zip(first + rest, full):
        assert torch.equal(a, b)  # the resumed run continues bit-identically


@pytest.mark.parametrize("auto_mark", [False, True])
def test_resume_mid_window_is_exact(auto_mark):
    """Checkpoint after 6 of 12 batches (windows of 4 batches: mid-window of epoch 1), resume in a fresh job."""
    kw = dict(env=None, output=ddl_amd.OutputSpec(copy_batches=True), order=ddl_amd.OrderSpec(shuffle="device",
                                                                                              seed=7),
              auto_mark=auto_mark)

    def run(n_batches, resume=None):
        rows, sd = [], None
        with ddl_amd.start(n_producers=3) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 3, **dict(kw, env=env),
                                               resume_state=resume)
            done = 0
            while dl.epoch < 3 and done < n_batches:
                for b in dl:
                    rows.append(torch.cat(b, 1).clone())
                    done += 1
                    if not auto_mark:
                        dl.mark(Marker.END_OF_BATCH)
                    if done == n_batches:
                        sd = dl.state_dict()
                        break
                else:
                    if not auto_mark:
                        dl.mark(Marker.END_OF_EPOCH)
                    continue
                break
            dl.close()
        return rows, sd

    head, sd = run(6)
    assert sd["epoch"] == 1 and sd["batch"] == 2 and sd["epoch_batch"] == 2  # mid-window
    tail, _ = run(10 ** 9, resume=sd)
    full, _ = run(10 ** 9)
    assert len(head) + len(tail) == len(full) == 12
    for a, b in zip(head + tail, full):
        assert torch.equal(a, b)


def test_producer_on_init_failure_is_reported():
    with pytest.raises(PeerDeathError, match="boom in on_init"):
        with ddl_amd.start(n_producers=2) as (env, conn):
            ddl_amd.DistributedDataLoader(FailingProducer(), 4, conn, 1, env=env)


def test_producer_crash_midrun_is_detected(monkeypatch):
    monkeypatch.setenv("DDL_FAULT_PRODUCER", "1:1:exit")
    with pytest.raises(PeerDeathError):
        with ddl_amd.start(n_producers=2, timeout_s=60) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(8, 4), 4, conn, 10, env=env)
            _epochs(dl, 10, collect=False)


def test_producer_exception_midrun_is_reported(monkeypatch):
    monkeypatch.setenv("DDL_FAULT_PRODUCER", "0:1:raise")
    with pytest.raises(PeerDeathError):
        with ddl_amd.start(n_producers=2, timeout_s=60) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(8, 4), 4, conn, 10, env=env)
            _epochs(dl, 10, collect=False)


def test_hung_producer_times_out(monkeypatch):
    monkeypatch.setenv("DDL_FAULT_PRODUCER", "0:1:hang")
    with pytest.raises(DDLTimeoutError):
        with ddl_amd.start(n_producers=1, timeout_s=3) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(8, 4), 4, conn, 5, env=env)
            _epochs(dl, 5, collect=False)


def test_window_smaller_than_batch_rejected():
    with pytest.raises(PeerDeathError, match="holds no batch"):
        with ddl_amd.start(n_producers=1) as (env, conn):
            ddl_amd.DistributedDataLoader(IdProducer(3, 4), 4, conn, 1, env=env)


def test_mismatched_producers_rejected():
    with pytest.raises(ShapeMismatchError):
        with ddl_amd.start(n_producers=2, env_overrides=None) as (env, conn):
            ddl_amd.DistributedDataLoader(_OddProducer(16, 4), 4, conn, 1, env=env)


class _OddProducer(IdProducer):
    def on_init(self, *a, **k):
        r = super().on_init(*a, **k)
        if self.producer_index == 1:
            r.splits = (1, self.width - 1)
        return r


def test_producer_preferred_slots(monkeypatch):
    """n_slots defaults to the producer's preferred_slots: 2 for whole-window refills (one slot refilled while
    the other is copied), 1 otherwise; an explicit n_slots wins."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    from ddl_amd.models.producers import ImageWindowProducer

    full, stamp = ImageWindowProducer(8, (3, 4, 4), "float32", refill="full"), ImageWindowProducer(8, (3, 4, 4))
    assert (full.preferred_slots, full.host_threads) == (2, 8)
    assert (stamp.preferred_slots, stamp.host_threads) == (1, 4)
    with ddl_amd.start(n_producers=1) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(full, 4, conn, 2, env=env)
        assert dl.n_slots == 2
        seen = [x[0].clone() for x in dl]
        assert len(seen) == 2
        dl.close()


def test_producers_exit_quickly_but_run_their_cleanup(monkeypatch, tmp_path):
    """Producer processes skip the interpreter teardown at their clean shutdown (os._exit after it): the
    loader's last epoch no longer waits ~0.8 s per producer; their atexit handlers still run, and a file the
    producer object held is flushed when the object is released; exit status 0."""
    import time

    from tests.helpers import AtexitProducer

    monkeypatch.setenv("DDL_DEVICE", "cpu")
    base = str(tmp_path / "p")
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(AtexitProducer(base, n=64, width=6), 16, conn, 2, env=env,
                                           auto_mark=True)
        for _ in range(2):
            for _b in dl:
                pass
        t0 = time.perf_counter()
        dl.close()
        took = time.perf_counter() - t0
        procs = list(conn.processes)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for i in range(2):
        assert open(f"{base}.atexit{i}").read() == "ran"
        assert open(f"{base}.log{i}").read() == "buffered"
    assert took < 5.0


def test_spare_connections_serve_later_loaders_and_unused_ones_exit_cleanly():
    """``start(spare_connections=)`` spawns more producer sets up front (before the GPU is touched): a second
    loader after the first runs on ``conn.spares[0]`` (its own producers, its own arena) and delivers every row
    exactly once; a spare that no loader used exits with status 0 at the end (no error report)."""
    with ddl_amd.start(n_producers=2, spare_connections=2) as (env, conn):
        assert len(conn.spares) == 2 and all(s.n_producers == 2 for s in conn.spares)
        first = ddl_amd.DistributedDataLoader(IdProducer(32, 4), 8, conn, 2, env=env)
        a = _epochs(first, 2)
        second = ddl_amd.DistributedDataLoader(IdProducer(48, 4), 8, conn.spares[0], 2, env=env)
        b = _epochs(second, 2)
        for rows, n in ((a, 32), (b, 48)):
            for ep in rows:
                assert sorted(ep[:, 2].tolist()) == list(range(n))  # column 2: the row id inside the window
        unused = conn.spares[1].processes
    assert all(p.exitcode == 0 for p in unused), [p.exitcode for p in unused]
