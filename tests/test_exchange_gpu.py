"""Global-shuffle exchange on the GPU path: RCCL process group, prefetch-stream
execution, gfx950 gather/scatter kernels (world size 1 on the single-GPU box;
multi-rank exchange semantics are covered over gloo in test_multirank_cpu)."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_env():
    import torch.distributed as dist

    from ddl_amd.types import DDLEnv
    from tests.mp_harness import free_port

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(free_port())})
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    env = DDLEnv(rank=0, world_size=1, device="cuda:0", backend="nccl", process_group=dist.group.WORLD,
                 control_group=dist.new_group(backend="gloo"))
    yield env
    dist.destroy_process_group()


def test_alltoall_exchange_on_device_conserves_window(rccl_env):
    from ddl_amd.parallel.shuffle import AllToAllGlobalShuffler

    n, row = 512, (3, 16, 16)
    win = torch.randint(0, 1 << 30, (n, *row), dtype=torch.int32, device="cuda")
    ref = win.clone()
    sh = AllToAllGlobalShuffler(rccl_env, 0.5, n, row, torch.int32, seed=3, device=win.device)
    assert sh.n_exchange == 256
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        sh(win.view(-1).view(torch.uint8), window=4)
    s.synchronize()
    assert torch.equal(win, ref)  # world 1: every row comes back to its own slot
    assert sh.calls == 1


@pytest.mark.parametrize("method", ["alltoall", "sendrecv_replace"])
def test_loader_with_exchange_enabled_on_gpu(rccl_env, monkeypatch, method):
    """The stager runs the exchange on its post-copy stream; batches stay exactly-once -- with the
    all-to-all and with the reference's two-partner pattern (``sendrecv_replace``: grouped isend / irecv,
    here to the rank itself) through RCCL."""
    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.parallel import launcher
    from tests.helpers import IdProducer

    conn = launcher.spawn_producers(ddl_amd.parallel.read_env(2), mode="thread")
    try:
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8), 16, conn, 4, 0.5, method, env=rccl_env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=2))
        assert dl._exchange_fn is not None and dl._stager.stream is not dl._stager.copy_stream
        for e in range(4):
            rows = []
            for i, (a, b) in enumerate(dl):
                rows.append(torch.cat([a, b], 1).cpu())
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
            rows = torch.cat(rows)
            assert sorted(rows[:, 2].tolist()) == list(range(64))
        assert dl._exchange_fn.calls == 4
    finally:
        conn.finalize()


def test_partial_epochs_with_exchange_keep_windows_intact(rccl_env):
    """Partial epochs skip windows: a skipped window is staged and exchanged but no batch reads it.
    Its buffer's free event must still follow that exchange, or the next copy into the buffer
    races the scatter; every delivered row must carry its own window's round."""
    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.parallel import launcher
    from tests.helpers import IdProducer

    P = 2
    conn = launcher.spawn_producers(ddl_amd.parallel.read_env(P), mode="thread")
    try:
        dl = ddl_amd.DistributedDataLoader(IdProducer(256, 8), 16, conn, 12, 0.5, "alltoall", env=rccl_env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=5, mode="split_along_epoch"))
        for e in range(12):
            w = dl.window
            for i, (a, b) in enumerate(dl):
                rows = torch.cat([a, b], 1).cpu()
                assert (rows[:, 1] == w % P).all() and (rows[:, 3] == w // P).all(), (e, i)
                dl.mark(Marker.END_OF_BATCH)
                if i == 2:
                    break  # partial epoch: the rest of this window and the epoch's next window are skipped
            dl.mark(Marker.END_OF_EPOCH)
        assert dl._exchange_fn.calls >= 12
    finally:
        conn.finalize()


def _exchange_run(env, dispatch, epochs=4, restore_at=None):
    """Rows of every batch of an exchange-on loader; with ``restore_at`` a live load_state_dict is done
    after that many batches (3 more are consumed first and then replayed)."""
    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.parallel import launcher
    from tests.helpers import IdProducer

    conn = launcher.spawn_producers(ddl_amd.parallel.read_env(3), mode="thread")
    out, sd, n = [], None, 0
    try:
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8), 16, conn, epochs, 0.5, "alltoall", env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(native_dispatch=dispatch),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=2))
        mode = dl.stats().get("native_dispatch", {}).get("mode") if dispatch else "python"
        while dl.epoch < epochs:
            for i in range(dl.epoch_batch, len(dl)):
                out.append(torch.cat([t.reshape(t.shape[0], -1) for t in dl[i]], 1).cpu())
                dl.mark(Marker.END_OF_BATCH)
                n += 1
                if restore_at is not None and n == restore_at:
                    sd = dl.state_dict()
                if sd is not None and n == restore_at + 3:
                    dl.load_state_dict(sd)
                    del out[restore_at:]
                    sd, restore_at = None, None
                    break
            else:
                dl.mark(Marker.END_OF_EPOCH)
        calls = dl._exchange_fn.calls
    finally:
        conn.finalize()
    return out, mode, calls


@pytest.mark.parametrize("dispatch", ["inline", "lookahead", "auto"])
def test_exchange_runs_on_the_native_engine(rccl_env, dispatch):
    """With the exchange on, batches come from the native engine (not the Python fallback) and are
    bit-identical to the Python dispatch path: the engine waits on the post-exchange ready event."""
    ref, mode_ref, calls_ref = _exchange_run(rccl_env, False)
    got, mode, calls = _exchange_run(rccl_env, dispatch)
    assert mode_ref == "python" and mode in ("inline", "lookahead", "window")
    if dispatch != "auto":
        assert mode == dispatch
    assert calls == calls_ref == 4 and len(got) == len(ref) == 16
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dispatch", ["auto", False])
def test_exchange_loader_live_load_state_dict(rccl_env, dispatch):
    """Live restore on an exchange-on loader: collectives restart at the checkpointed window and the
    delivered batches equal the uninterrupted run."""
    ref, _, _ = _exchange_run(rccl_env, dispatch)
    for at in (2, 5):
        got, _, _ = _exchange_run(rccl_env, dispatch, restore_at=at)
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)


@pytest.mark.parametrize("dispatch", ["auto", False])
def test_exchange_stuck_copy_raises_within_the_timeout(rccl_env, dispatch):
    """With the exchange on, the consumer host-waits for window w+1's copy before it enqueues w+1's
    all-to-all (direct DMA: no HIP event follows the copy). That wait is bounded too: a copy whose completion
    signal never drops (fault injection) raises DDLTimeoutError naming the window within the loader's
    timeout, and close() returns."""
    import time

    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.exceptions import DDLTimeoutError
    from ddl_amd.parallel import launcher
    from tests.helpers import IdProducer

    conn = launcher.spawn_producers(ddl_amd.parallel.read_env(2), mode="thread")
    try:
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8), 16, conn, 8, 0.5, "alltoall", env=rccl_env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2, timeout_s=3.0,
                                                                       native_dispatch=dispatch),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=2))
        if not dl._stager.direct_dma:
            pytest.skip("no direct DMA here")
        dl._stager._native.inject_stuck_copy(4)  # not staged yet: the 3-buffer ring holds windows 0..2
        t0 = time.monotonic()
        with pytest.raises(DDLTimeoutError, match="window 4"):
            for _ in range(8):
                for _ in dl:
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)
        assert time.monotonic() - t0 < 3.0 + 8.0
        t1 = time.monotonic()
        dl.close()
        assert time.monotonic() - t1 < 15.0
    finally:
        conn.finalize()
