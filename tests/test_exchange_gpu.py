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


def test_loader_with_exchange_enabled_on_gpu(rccl_env, monkeypatch):
    """The stager runs the exchange on its post-copy stream; batches stay exactly-once."""
    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.parallel import launcher
    from tests.helpers import IdProducer

    conn = launcher.spawn_producers(ddl_amd.parallel.read_env(2), mode="thread")
    try:
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8), 16, conn, 4, 0.5, "alltoall", env=rccl_env,
                                           shuffle="device", copy_batches=True, seed=2)
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
                                           shuffle="device", copy_batches=True, seed=5, mode="split_along_epoch")
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
