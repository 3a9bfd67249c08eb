"""Cross-cutting layer: hook dispatch, lazy logging, typed errors, env parsing, NUMA."""

import logging
import os

import pytest

from ddl_amd.exceptions import DoesNotMatchError, TopologyError
from ddl_amd.parallel.env import read_env
from ddl_amd.parallel.shuffle import derangement_partners
from ddl_amd.utils.callbacks import execute_callbacks
from ddl_amd.utils.logging import for_all_methods, with_logging


class _A:
    def __init__(self, log):
        self.log = log

    def on_init(self, **kw):
        self.log.append(("A", kw["x"]))
        return "from-A"

    def global_shuffle(self, **kw):
        self.log.append("A-shuffle")


class _B:
    def __init__(self, log):
        self.log = log

    def on_init(self, **kw):
        self.log.append(("B", kw["x"]))
        return "from-B"

    def global_shuffle(self, **kw):
        self.log.append("B-shuffle")


def test_every_callback_runs_in_order():
    log = []
    ret = execute_callbacks("on_init", [_A(log), _B(log)], x=1)
    assert log == [("A", 1), ("B", 1)]  # reference runs only callbacks[0] (ddl/utils.py:22)
    assert ret == "from-A"
    execute_callbacks("global_shuffle", [_A(log), object(), _B(log)])
    assert log[-2:] == ["A-shuffle", "B-shuffle"]
    assert execute_callbacks("missing_hook", [_A(log)]) is None


class _Loud:
    def __init__(self):
        self.n = 0

    def __repr__(self):
        self.n += 1
        return "loud"


def test_with_logging_is_lazy(caplog):
    @with_logging
    def f(a):
        return 3

    loud = _Loud()
    logging.getLogger("ddl_amd").setLevel(logging.INFO)
    assert f(loud) == 3
    assert loud.n == 0  # reference builds repr() eagerly on every call (ddl/utils.py:28-30)
    logging.getLogger("ddl_amd").setLevel(logging.DEBUG)
    with caplog.at_level(logging.DEBUG, logger="ddl_amd"):
        f(loud)
    assert loud.n == 1 and "loud" in caplog.text
    logging.getLogger("ddl_amd").setLevel(logging.WARNING)


def test_with_logging_reraises(caplog):
    @with_logging
    def g():
        raise KeyError("x")

    with pytest.raises(KeyError):
        g()
    assert "exception raised" in caplog.text


def test_for_all_methods_no_double_wrap():
    calls = []

    def deco(fn):
        calls.append(fn.__name__)
        return fn

    @for_all_methods(deco, exclude="skip")
    class C:
        def a(self):
            pass

        def skip(self):
            pass

        @staticmethod
        def s():
            pass

        @property
        def p(self):
            return 1

    assert sorted(calls) == ["__init__"] or sorted(calls) == ["a"]


def test_does_not_match_error_constructor():
    e = DoesNotMatchError((1, 2), "mismatch")  # reference typo __init (ddl/exceptions.py:2)
    assert e.value == (1, 2) and e.message == "mismatch" and str(e) == "mismatch"


def test_read_env_torchrun(monkeypatch):
    for k in ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID", "SLURM_NTASKS_PER_NODE", "SLURM_NNODES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("RANK", "5")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    env = read_env(2)
    assert (env.rank, env.world_size, env.local_rank, env.local_world_size, env.node_rank) == (5, 8, 1, 4, 1)
    assert env.n_instances == 8 and env.n_producers == 2


def test_read_env_slurm_fallback(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("SLURM_PROCID", "3")
    monkeypatch.setenv("SLURM_NTASKS", "4")
    monkeypatch.setenv("SLURM_LOCALID", "3")
    monkeypatch.setenv("SLURM_NNODES", "1")
    monkeypatch.setenv("DDL_PRODUCERS_PER_RANK", "5")
    env = read_env()
    assert (env.rank, env.world_size, env.local_rank, env.local_world_size, env.n_producers) == (3, 4, 3, 4, 5)


@pytest.mark.parametrize("bad", [{"RANK": "4", "WORLD_SIZE": "4"}, {"RANK": "0", "WORLD_SIZE": "6", "LOCAL_WORLD_SIZE": "4"},
                                 {"RANK": "x"}])
def test_read_env_errors(monkeypatch, bad):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in bad.items():
        monkeypatch.setenv(k, v)
    with pytest.raises(TopologyError):
        read_env(1)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
def test_derangement_partners_consistent(n):
    import numpy as np

    pairs = [derangement_partners(n, r, np.random.default_rng([0, 4])) for r in range(n)]
    send = [p[0] for p in pairs]
    recv = [p[1] for p in pairs]
    for r in range(n):
        assert recv[send[r]] == r  # my receiver receives from me
        if n > 2:
            assert send[r] != r and send[r] != recv[r]  # no self, no 2-cycle


def test_numa_helpers_do_not_fail():
    from ddl_amd.utils import numa

    numa.visible_gpu_render_minors()
    assert numa.node_cpus(0) or True
    assert numa.bind_to_gpu_numa(0) in (None, 0, 1, 2, 3, 4, 5, 6, 7)


def test_cpu_slices_partition_a_node(monkeypatch):
    """4 GPUs on node 0 with 32 CPUs: each local rank gets a disjoint 8-CPU slice; the consumer keeps 4 of
    its slice and its producers share the other 4 only when there is room for both."""
    from ddl_amd.utils import numa

    monkeypatch.setattr(numa, "gpu_numa_node", lambda i: 0 if i < 4 else 1)
    monkeypatch.setattr(numa, "node_cpus", lambda n: set(range(32)) if n == 0 else set(range(32, 64)))
    allowed = set(range(64))
    slices = [numa.rank_cpu_slice(i, 8, allowed) for i in range(8)]
    assert [n for n, _ in slices] == [0, 0, 0, 0, 1, 1, 1, 1]
    for i, (_, c) in enumerate(slices):
        assert len(c) == 8 and c == set(range(8 * i, 8 * i + 8))
    cons, prod = numa.split_consumer_producers(slices[1][1], 2)
    assert cons == {8, 9, 10, 11} and prod == {12, 13, 14, 15}
    cons, prod = numa.split_consumer_producers(slices[1][1], 3)  # 4 + 2*3 > 8: no split
    assert cons == prod == slices[1][1]
    assert numa.rank_cpu_slice(0, 1, allowed) == (0, set(range(32)))  # alone on the node: all of it


def test_normalize_columns_cpu_reference():
    import numpy as np
    import torch

    from ddl_amd import ops

    x = torch.randn(1000, 5) * 3 + 2
    y = ops.normalize_columns(x, "standard")
    np.testing.assert_allclose(y.mean(0).numpy(), 0, atol=1e-5)
    np.testing.assert_allclose(y.std(0, unbiased=False).numpy(), 1, atol=1e-4)
    z = ops.normalize_columns(x, "minmax")
    np.testing.assert_allclose(z.min(0).values.numpy(), -1, atol=1e-5)
    np.testing.assert_allclose(z.max(0).values.numpy(), 1, atol=1e-5)


def test_metrics_writer(tmp_path):
    import json

    import ddl_amd
    from ddl_amd import Marker
    from ddl_amd.utils.metrics import MetricsWriter
    from tests.helpers import IdProducer

    path = tmp_path / "m" / "metrics.jsonl"
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(16, 4), 4, conn, 2, env=env)
        mw = MetricsWriter(dl, str(path), interval_s=0.0)
        for _ in range(2):
            for i, _b in enumerate(dl):
                dl.mark(Marker.END_OF_BATCH)
                mw.step()
            dl.mark(Marker.END_OF_EPOCH)
        rec = mw.flush()
    lines = path.read_text().splitlines()
    assert len(lines) >= 8
    last = json.loads(lines[-1])
    assert last["batches"] == 8 and last["samples"] == 32 and "consumer_wait_s" in last
    assert rec["producer_rounds"] and len(rec["producer_rounds"]) == 2


def _trace_idle():
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(__file__), "..", "tools", "trace_idle.py")
    spec = importlib.util.spec_from_file_location("trace_idle", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_trace_idle_union_and_gaps():
    ti = _trace_idle()
    busy, gaps = ti.union_ns([(10, 20), (15, 30), (50, 60), (95, 200)], 0, 100)
    assert busy == 20 + 10 + 5
    assert gaps == [(0, 10), (30, 50), (60, 95)]


def test_trace_idle_analyse_regions():
    ti = _trace_idle()

    def k(a, b, name):
        return {"Kernel_Name": name, "Start_Timestamp": str(a), "End_Timestamp": str(b)}

    kernels = [k(100, 400, "move_rows_chunked<...>"), k(300, 600, "Cijk_gemm"), k(700, 1000, "checksum_acc")]
    copies = [{"Start_Timestamp": "0", "End_Timestamp": "500"}]
    markers = [{"Function": "bench.phase2", "Start_Timestamp": "0", "End_Timestamp": "1000"},
               {"Function": "ddl.consumer.batch", "Start_Timestamp": "5", "End_Timestamp": "6"}]
    r = ti.analyse(kernels, copies, markers)["bench.phase2"]
    assert r["device_idle_pct"] == 20.0  # busy 100..600 and 700..1000 of 0..1000
    assert r["loader_kernel_pct"] == 60.0
    assert r["copy_busy_pct"] == 50.0
    assert r["kernel_dispatches"] == 3


def test_numa_local_source_and_memory_binding():
    """Per-NUMA-node replica of a node-shared array: created by the node's first rank, bound to the node
    with mbind, filled; pages report the node (move_pages)."""
    import numpy as np
    import torch

    from ddl_amd.models import numa_local_source
    from ddl_amd.types import DDLEnv

    env = DDLEnv(rank=0, world_size=1, local_rank=0, local_world_size=1)
    name = f"ddl_amd_numa_t{np.random.randint(1 << 30)}"
    src, node, created = numa_local_source(name, 64, (16,), "float32", env,
                                           fill=lambda t: t.copy_(torch.arange(64 * 16.0).view(64, 16)))
    try:
        assert created and src.name.startswith(name + "_numa")
        assert torch.equal(src.tensor().view(-1), torch.arange(64 * 16.0))
        assert src.bind_to_node(0) == 0  # node 0 exists on every Linux host
        pages = src.page_nodes(8)
        assert pages and all(p == 0 for p in pages)
    finally:
        src.close()


def test_partition_after_spawn_leaves_the_consumer_process_alone():
    """The consumer is the user's training process: the CPU split moves only the producers (ADVICE r3:
    confining the whole process to 4 CPUs also confined torch's intra-op pool and the user's threads)."""
    import subprocess
    import sys

    from ddl_amd.utils import numa

    mine = os.sched_getaffinity(0)
    if len(mine) < 6:
        pytest.skip("needs >= 6 CPUs")
    child = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        layout = numa.partition_after_spawn([child.pid], 1)
        assert layout is not None
        assert os.sched_getaffinity(0) == mine
        assert set(layout["consumer_cpus"]) == mine
        assert os.sched_getaffinity(child.pid) == set(layout["producer_cpus"])
        assert not set(layout["consumer_reserved_cpus"]) & set(layout["producer_cpus"])
    finally:
        child.kill()
        child.wait()


def test_compute_idle_meter_gap_distribution():
    """result() reports the idle and where it sits (per-boundary gaps), from the events' timestamps."""
    from ddl_amd.utils.tracing import ComputeIdleMeter

    class Ev:
        def __init__(self, t_ms):
            self.t = t_ms

        def elapsed_time(self, other):
            return other.t - self.t

        def synchronize(self):
            pass

    m = ComputeIdleMeter.__new__(ComputeIdleMeter)
    # 100 steps of 1 ms; 10 us gaps, except one 1 ms stall after step 50
    t, pairs = 0.0, []
    for i in range(100):
        pairs.append((Ev(t), Ev(t + 1.0)))
        t += 1.0 + (1.0 if i == 50 else 0.01)
    m._pairs = pairs
    r = m.result()
    assert r["steps"] == 100 and abs(r["busy_ms"] - 100.0) < 1e-9
    g = r["gaps_us"]
    assert abs(g["p50"] - 10.0) < 0.1 and abs(g["max"] - 1000.0) < 0.1
    assert abs(g["top1pct_share"] - 1000.0 / (1000.0 + 98 * 10.0)) < 1e-3
    assert abs(r["gpu_idle_pct"] - 100.0 * (1.0 - 100.0 / (100.0 + 1.0 + 0.98))) < 1e-6


def test_one_gpu_per_rank_is_enforced(monkeypatch):
    """More ranks on a node than visible GPUs, or a second rank of the job on a GPU (a per-job flock on its PCI
    bus ID), is a TopologyError -- unless DDL_REHEARSAL=1 labels the run a rehearsal."""
    import os

    from ddl_amd.exceptions import TopologyError
    from ddl_amd.parallel import env as env_mod
    from ddl_amd.types import DDLEnv

    for v in env_mod._VISIBILITY_VARS:
        monkeypatch.delenv(v, raising=False)
    monkeypatch.delenv("DDL_REHEARSAL", raising=False)
    e = DDLEnv(rank=1, world_size=8, local_rank=1, local_world_size=8, hostname="h")
    env_mod.check_device_count(e, 8)
    with pytest.raises(TopologyError, match="share a device"):
        env_mod.check_device_count(e, 1)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")  # per-task masks: the bus-ID checks decide instead
    env_mod.check_device_count(e, 1)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("DDL_REHEARSAL", "1")
    env_mod.check_device_count(e, 1)
    monkeypatch.delenv("DDL_REHEARSAL")

    bus = f"0000:{os.getpid() % 251:02x}:1f"
    monkeypatch.setattr(env_mod, "device_identity", lambda device: {"pci_bus_id": bus})
    monkeypatch.setenv("MASTER_PORT", str(40000 + os.getpid() % 20000))
    env_mod.claim_device(DDLEnv(rank=0, world_size=2, device="cuda:0"))
    fd = env_mod._CLAIMED.pop(bus)  # as if rank 0 were another process still holding the claim
    try:
        with pytest.raises(TopologyError, match=r"rank 1 and rank 0 \(pid"):
            env_mod.claim_device(DDLEnv(rank=1, world_size=2, device="cuda:0"))
        monkeypatch.setenv("DDL_REHEARSAL", "1")
        env_mod.claim_device(DDLEnv(rank=1, world_size=2, device="cuda:0"))  # a rehearsal may share
    finally:
        os.close(fd)
