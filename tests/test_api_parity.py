"""The reference's class and protocol names beyond its five exports."""

import pytest
import torch

import ddl_amd
from ddl_amd import Marker
from ddl_amd.connection import Connection, ProducerConnection
from ddl_amd.dataloader import DistributedDataloaderABC
from ddl_amd.datapusher import DataPusher, DataPusherABC
from ddl_amd.exceptions import TopologyError
from ddl_amd.parallel import init_mpi
from ddl_amd.types import DDLEnv, MPI_Env
from tests.helpers import IdProducer


@pytest.fixture(autouse=True)
def _host_path(monkeypatch):
    monkeypatch.setenv("DDL_DEVICE", "cpu")


def test_abstract_bases_carry_the_reference_method_names():
    # reference ddl/mpi_dataloader.py:31-103 and ddl/datapusher.py:22-41
    assert DistributedDataloaderABC.__abstractmethods__ == {
        "__len__", "__getitem__", "_advance_to_next_producer", "_finalize", "_start_access_epoch",
        "_end_access_epoch", "_can_continue", "mark"}
    assert DataPusherABC.__abstractmethods__ == {"push_data", "_start_access_epoch", "_end_access_epoch", "sync",
                                                 "_finalize"}
    assert issubclass(ddl_amd.DistributedDataLoader, DistributedDataloaderABC)
    assert issubclass(DataPusher, DataPusherABC)
    assert not ddl_amd.DistributedDataLoader.__abstractmethods__ and not DataPusher.__abstractmethods__
    for cls in (Connection, ProducerConnection):  # Win.Sync barrier names (ddl/connection.py:61-63, 144-151)
        assert callable(cls.sync) and callable(cls._sync)


def test_mpi_env_alias_and_communicator_properties():
    assert MPI_Env is DDLEnv
    env = DDLEnv(rank=1, world_size=2, process_group="pg")
    assert env.comm_global == "pg" and env.comm_nth_pusher == "pg" and env.comm_per_gpu_shm is None
    assert env.n_instances == 2 and env.color == 1


def test_init_mpi_single_rank_and_mismatch(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    env = init_mpi(1, n_producers=0)
    assert env.world_size == 1 and env.device == "cpu" and env.comm_global is None
    with pytest.raises(TopologyError):
        init_mpi(8)


def test_reference_protocol_methods_drive_the_window_round_robin():
    """_end_access_epoch / _advance_to_next_producer / _start_access_epoch, called by hand, move the
    consumer to the next producer's window exactly as mark(END_OF_BATCH) does at a window's end
    (reference ddl/mpi_dataloader.py:220-227)."""
    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(8, 4), 4, conn, 1, env=env,
                                           order=ddl_amd.OrderSpec(mode="split_along_epoch"))
        assert len(dl) == 6 and dl.target_rank == 1
        _, rest = dl[0]
        dl.mark(Marker.END_OF_BATCH)
        dl._end_access_epoch()
        dl._advance_to_next_producer()
        dl._start_access_epoch()
        assert dl.target_rank == 2 and dl.window == 1
        ids, _ = dl[1]  # epoch index 1 = first batch of producer 2's window (window 0 skipped its batch 1)
        assert ids[:, 1].unique().tolist() == [1] and ids[:, 0].tolist() == [0, 0, 0, 0]
        assert dl._can_continue()
        dl.close()
        assert dl._finalized


def test_constructor_keeps_the_reference_eight_and_groups_the_rest():
    """The reference's eight arguments come first, positionally (reference ddl/mpi_dataloader.py:108-118);
    everything the MI355X loader adds is keyword-only, and its ~20 options live in three records."""
    import inspect

    params = list(inspect.signature(ddl_amd.DistributedDataLoader.__init__).parameters.values())[1:]
    positional = [p.name for p in params if p.kind is p.POSITIONAL_OR_KEYWORD]
    assert positional == ["producer_function", "batch_size", "connection", "n_epochs", "fraction_exchange",
                          "exchange_method", "instance_idx", "n_instances"]
    keyword = [p.name for p in params if p.kind is p.KEYWORD_ONLY]
    assert keyword == ["env", "device", "output", "staging", "order", "auto_mark", "resume_state", "debug_checksum"]


def test_specs_validate_and_legacy_keywords_are_deprecated_aliases():
    from ddl_amd.specs import OrderSpec, OutputSpec, StagingSpec, resolve

    with pytest.raises(ValueError):
        OrderSpec(mode="bogus")
    with pytest.raises(ValueError):
        OutputSpec(augment={"bogus": 1})
    with pytest.raises(ValueError):
        StagingSpec(native_dispatch="sideways")
    with pytest.raises(ValueError):
        StagingSpec(max_ahead=-1)
    with pytest.raises(TypeError):
        resolve(None, None, None, {"not_an_option": 1})
    with pytest.warns(DeprecationWarning) as rec:
        out, stg, odr = resolve(None, StagingSpec(prefetch_depth=2), None, {"seed": 5, "out_dtype": torch.bfloat16})
    msgs = sorted(str(w.message) for w in rec)
    assert any("order=OrderSpec(seed=...)" in m for m in msgs) and any("output=OutputSpec(dtype=...)" in m for m in msgs)
    assert odr.seed == 5 and out.dtype is torch.bfloat16 and stg.prefetch_depth == 2
    with pytest.raises(dataclasses_frozen_error()):
        odr.seed = 1  # records are frozen


def dataclasses_frozen_error():
    import dataclasses

    return dataclasses.FrozenInstanceError


def test_spec_and_legacy_construction_deliver_the_same_batches():
    def run(**kw):
        with ddl_amd.start(n_producers=2) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 2, env=env, auto_mark=True, **kw)
            got = [torch.cat(b, 1).clone() for _ in range(2) for b in dl]
            opts = (dl.seed, dl.shuffle, dl.mode, dl.copy_batches, dl.prefetch_depth)
            dl.close()
        return got, opts

    new, o1 = run(order=ddl_amd.OrderSpec(shuffle="device", seed=9, mode="split_along_epoch"),
                  staging=ddl_amd.StagingSpec(prefetch_depth=2))
    with pytest.warns(DeprecationWarning):
        old, o2 = run(shuffle="device", seed=9, mode="split_along_epoch", prefetch_depth=2)
    assert o1 == o2 == (9, "device", "split_along_epoch", True, 2)
    assert len(new) == len(old) > 0 and all(torch.equal(a, b) for a, b in zip(new, old))
