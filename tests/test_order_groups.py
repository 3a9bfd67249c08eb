"""The one-communicator invariant (``ddl_amd/parallel/order.py``), checked on process groups.

The reference runs its exchange on a communicator of its own (``comm_nth_pusher``, reference
ddl/ddl_env.py:74-81) next to the trainer's; with RCCL two communicators on two streams can deadlock
across ranks, so here every loader collective (window exchange, resident all-to-all, the resident
shard scatter's point-to-point batches) and the DDP hook must be issued on ``env.process_group``
itself. These tests (gloo, 2 ranks) assert that every recorded collective used that one group, and
that a loader collective on any other group raises instead of running.
"""

import numpy as np
import pytest
import torch

from tests.mp_harness import run_ranks


def _all_on_dp_group(rank, world, name):
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.models import SharedArraySource
    from ddl_amd.models.trainstep import TrainStep
    from ddl_amd.parallel.order import LEDGER, check_same_order, group_id
    from ddl_amd.resident import ResidentGlobalLoader
    from tests.helpers import IdProducer

    LEDGER.clear()
    LEDGER.enable(True)
    src = SharedArraySource(name, 96, (3,), "int64") if rank == 0 else None
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(32, 6), 8, conn, 2, 0.5, "alltoall", env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           order=ddl_amd.OrderSpec(seed=1))
        step = TrainStep(torch.device("cpu"), dim=8, depth=1, process_group=env.process_group)
        for _ in range(2):
            for a, b in dl:
                step(torch.ones(a.shape[0], 3, 16, 16) * a[:, :1, None, None].float())
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
        res = ResidentGlobalLoader(src, 24, env, seed=3, n_epochs=1, scatter_from=0, chunk_bytes=24 * 8)
        n_res = sum(1 for _ in res)
        order = check_same_order(env.control_group)
        groups = set(LEDGER.groups)
        want = group_id(env.process_group)
        dist.barrier(group=env.control_group)
    LEDGER.enable(False)
    return order, groups, want, n_res


def test_every_loader_collective_and_ddp_use_the_dp_group():
    from ddl_amd.models import SharedArraySource

    name = f"ddl_amd_order_{np.random.randint(1 << 30)}"
    src = SharedArraySource(name, 96, (3,), "int64", create=True)
    try:
        src.tensor().view(-1).copy_(torch.arange(96 * 3))
        res = run_ranks(_all_on_dp_group, 2, name, timeout=240)
    finally:
        src.close()
    for order, groups, want, n_res in res:
        assert order["same_order"] is True and order["groups"] == 1
        assert groups == {want}
        kinds = order["by_kind"]
        assert kinds["loader.exchange"] >= 2 and kinds["ddp.allreduce"] >= 2
        assert kinds["resident.all_to_all"] == n_res > 0 and kinds["resident.bringup"] == 1


def _mismatched_group(rank, world):
    import torch.distributed as dist

    import ddl_amd
    from ddl_amd.exceptions import CommunicatorMismatchError
    from ddl_amd.parallel.order import check_group
    from ddl_amd.parallel.shuffle import AllToAllGlobalShuffler

    with ddl_amd.start(n_producers=0) as (env, _):
        other = dist.new_group(backend="gloo")  # same ranks, another communicator
        raised = []
        try:
            AllToAllGlobalShuffler(env, 0.5, 64, (4,), torch.int32, 0, torch.device("cpu"), group=other)
        except CommunicatorMismatchError:
            raised.append("exchange")
        try:
            check_group(env, other, "resident.scatter_p2p")
        except CommunicatorMismatchError:
            raised.append("p2p")
        # the right group passes, and an exchange built on it really runs
        sh = AllToAllGlobalShuffler(env, 0.5, 64, (4,), torch.int32, 0, torch.device("cpu"))
        win = torch.arange(64 * 4, dtype=torch.int32).reshape(64, 4) + 1000 * rank
        sh(win.view(-1).view(torch.uint8), window=0)
        dist.barrier(group=env.control_group)
    return raised, int((win // 1000 != rank).sum())


def test_loader_collective_on_another_group_raises():
    res = run_ranks(_mismatched_group, 2, timeout=120)
    for raised, foreign in res:
        assert raised == ["exchange", "p2p"]
        assert foreign > 0  # the exchange on the DP group traded rows


def test_check_group_rejects_none_and_foreign_objects():
    from ddl_amd.exceptions import CommunicatorMismatchError
    from ddl_amd.parallel.order import check_group, issue
    from ddl_amd.types import DDLEnv

    env = DDLEnv(rank=0, world_size=1, process_group=object())
    check_group(env, env.process_group, "ok")
    for bad in (None, object()):
        with pytest.raises(CommunicatorMismatchError, match="DP process group"):
            issue(env, bad, "loader.exchange", 0)
