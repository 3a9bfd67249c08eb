"""Several DP ranks on the GPU box's one card: the multi-process device data path on hardware.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected", ``archive/profiles/r1_rccl_probe``), so
these runs build the DP group on gloo (``DDL_BACKEND=gloo``; gloo's all-to-all and all-reduce
take device tensors and bounce them through host memory). Everything else is the production
path of each rank: its own producer processes and pinned arena, H2D staging on the copy
streams, the window exchange on the post-copy stream, the gfx950 gather/permute kernels and a
DDP train step -- with two or four of them sharing the card. The reference's exchange this
replaces is ``/root/reference/ddl/shuffle.py:92-108``; the CPU versions of these checks are in
``test_multirank_cpu.py`` and ``test_examples.py``.
"""

import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests.mp_harness import free_port, run_ranks

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# "" = not forced to the CPU; several ranks share the one card of a gpurun box: a labelled rehearsal
GPU_GLOO = {"DDL_DEVICE": "", "DDL_BACKEND": "gloo", "DDL_REHEARSAL": "1"}


def _exchange_rank_gpu(rank, world, method, fraction, slow=0.0):
    import time

    import ddl_amd
    from ddl_amd import Marker
    from tests.helpers import IdProducer

    eps = []
    with ddl_amd.start(n_producers=2) as (env, conn):
        assert env.device.startswith("cuda"), env.device
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 6), 16, conn, 3, fraction, method, env=env,
                                           device=torch.device(env.device),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2),
                                           order=ddl_amd.OrderSpec(seed=1))
        assert dl._exchange_fn is not None
        direct = dl.stats()["direct_dma"]
        for _ in range(3):
            rows = []
            for a, b in dl:
                assert a.is_cuda and b.is_cuda
                rows.append(torch.cat([a, b], 1).cpu())
                if slow:  # the consumer is the bottleneck: the ring fills, the stager waits on free events
                    time.sleep(slow)
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
            eps.append(torch.cat(rows).numpy())
        n_ex = dl._exchange_fn.n_exchange
        dl.close()
    return eps, n_ex, direct


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,slow", [(2, 0.0), (4, 0.0), (2, 0.01)])
def test_exchange_conserves_rows_on_device(world, slow):
    """The all-to-all window exchange between ranks whose windows live in HBM, on direct-DMA staging (the
    consumer host-waits each copy's completion signal before it enqueues the exchange), with a fast and a
    slow consumer: every (rank, producer, row) of every round is delivered exactly once over all ranks, and
    each rank holds exactly the foreign rows the exchange plan says."""
    res = run_ranks(_exchange_rank_gpu, world, "alltoall", 0.5, slow, timeout=200, env=GPU_GLOO)
    assert all(r[2] for r in res), "direct-DMA staging not in use"
    n_ex = res[0][1]
    assert n_ex > 0
    for e in range(3):
        all_rows = np.concatenate([r[0][e] for r in res])
        keys = {tuple(x) for x in all_rows[:, :3].tolist()}
        assert len(keys) == len(all_rows) == world * 64  # an epoch is one 64-row window per rank
        for r in range(world):
            mine = res[r][0][e]
            assert (mine[:, 0] != r).sum() == n_ex - n_ex // world  # the chunk for self stays


def _run_bench(n, launch, extra=()):
    args = [os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "24", "--warmup", "6",
            "--idle-steps", "6", *extra]
    env = dict(os.environ, PYTHONPATH=REPO, **GPU_GLOO)
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args]
    else:
        cmd = [sys.executable, *args]
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(240)
@pytest.mark.parametrize("n,launch", [(2, "torchrun"), (2, "self")])
def test_bench_multirank_device_path(n, launch):
    """bench.py at N ranks on the card: the driver's torchrun line and the self-launch both give one
    JSON line with n_gpus = N; every rank moved its windows H2D inside the timed region, ran the
    window exchange, and issued loader exchanges and DDP all-reduces in one cross-rank order."""
    out = _run_bench(n, launch)
    assert out["n_gpus"] == n and out["config"]["parallelism"] == f"dp{n}" and out["value"] > 0
    assert out["config"]["exchange_fraction"] == 0.5 and out["phase2_error"] is None
    order = out["collective_order"]
    assert order["same_order"] is True and order["groups"] == 1 and order["by_kind"]["ddp.allreduce"] > 0
    assert order["by_kind"]["loader.exchange"] > 0
    assert len(out["per_rank"]) == n
    for r in out["per_rank"]:
        assert r["h2d_bytes_timed"] > 0 and r["exchange_calls"] > 0 and r["rccl_bytes"] > 0
        # the exchange-on N > 1 point runs the same native batch engine as N = 1 (not the Python path)
        assert r["dispatch"]["mode"] in ("inline", "lookahead", "window"), r["dispatch"]
        assert r["dispatch"]["host_us_per_batch"]["get"] > 0
    assert out["config"]["dispatch"] == out["per_rank"][0]["dispatch"]["mode"]
    assert out["indexed"] and "error" not in out["indexed"] and out["indexed"]["value"] > 0
    # phase 3 (loader pressure) ran on all three paths, in step on every rank
    for sub in (out, out["indexed"], out["indexed"]["zero_copy"]):
        assert sub["pressure"] and "error" not in sub["pressure"], sub["pressure"]
        assert sub["gpu_idle_pct_r090"] is not None
    # the line labels itself: gloo ranks sharing one card, a rehearsal (not an N-GPU RCCL measurement)
    d = out["dist"]
    assert d["backend"] == "gloo" and d["group_size"] == n and d["distinct_gpus"] == 1
    assert d["rehearsal"] is True and d["verified"] is False and len(d["problems"]) >= 2
    assert all(r_["alltoall"]["data_ok"] for r_ in d["ranks"])
    for r in out["per_rank"]:
        w = r["exchange_issue_wait_timed"]
        assert w["exchange_issue_wait_n"] > 0 and w["exchange_issue_wait_p99_ms"] >= w["exchange_issue_wait_p50_ms"]


@pytest.mark.timeout(120)
def test_ranks_sharing_the_card_are_refused_without_rehearsal():
    """Two ranks on one GPU without DDL_REHEARSAL: the layout is refused at start (TopologyError: more ranks
    than visible GPUs), bench exits non-zero and prints no JSON line -- no silent device sharing."""
    args = [os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1", "--idle-steps", "0",
            "--pressure-ratio", "0", "--order", "window"]
    env = {k: v for k, v in os.environ.items() if k not in ("DDL_REHEARSAL", "DDL_BACKEND", "WORLD_SIZE", "RANK",
                                                            "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=REPO, DDL_DEVICE="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "TopologyError" in r.stderr and "share a device" in r.stderr


@pytest.mark.timeout(240)
def test_killed_rank_on_the_card_ends_the_job():
    """Two ranks on the card streaming a device loader with the exchange on; rank 1 is SIGKILLed mid-epoch
    (H2D copies, kernels and collectives in flight). Its death watch publishes the abort; rank 0 -- blocked
    in or heading into the next exchange -- exits with the peer-abort status (or 1 if the collective's own
    error reaches it first) within seconds, with no leftover processes."""
    import signal
    import time

    from ddl_amd.parallel.abort import PEER_ABORT_EXIT

    script = os.path.join(REPO, "tests", "abort_rank.py")
    port = str(free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, PYTHONPATH=REPO, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=port, **GPU_GLOO)
        procs.append(subprocess.Popen([sys.executable, script, "--gpu-loader", "--kill-rank", "1",
                                       "--peer-timeout", "60"], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, start_new_session=True))
    t0 = time.monotonic()
    try:
        while time.monotonic() - t0 < 150 and any(p.poll() is None for p in procs):
            time.sleep(0.1)
        took = time.monotonic() - t0
        codes = [p.poll() for p in procs]
    finally:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)  # the rank and its helpers (producers, death watch)
            except ProcessLookupError:
                pass
        outs = [p.communicate(timeout=30) for p in procs]
    assert "killing itself mid-epoch on cuda" in outs[1][0], outs[1][1][-2000:]
    assert codes[1] == -signal.SIGKILL, codes
    assert codes[0] in (PEER_ABORT_EXIT, 1), (codes, outs[0][1][-2000:])
    assert "died without a clean shutdown" in outs[0][1] or codes[0] == 1, outs[0][1][-2000:]
    assert took < 120, took


def _resident_rank_gpu(rank, world, name, n, gb, replicate, scatter):
    import numpy as np

    import ddl_amd
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    src = SharedArraySource(name, n, (3, 8, 8), "uint8") if (rank == 0 or not scatter) else None
    with ddl_amd.start(n_producers=0) as (env, _):
        dl = ResidentGlobalLoader(src, gb, env, seed=4, n_epochs=1, replicate=replicate,
                                  scatter_from=0 if scatter else None, chunk_bytes=192 * 37)
        assert dl.shard.is_cuda and dl.replicated == replicate
        ids = [b[:, 0, 0, 0].to(torch.int64).cpu().numpy() for b in dl]
        st = dl.stats()
        dl.close()
        return np.stack(ids), st["bytes_exchanged"], st["bytes_replicated"]


@pytest.mark.timeout(200)
@pytest.mark.parametrize("replicate,scatter", [(True, False), (True, True), (False, False)])
def test_resident_layouts_on_the_card(replicate, scatter):
    """The HBM-resident loader's GPU path at W = 2 (gloo on one card): replicated (all-gather bring-up, or
    scatter + all-gather from one holder) and sharded layouts deliver the same union order -- global batch g of
    the epoch permutation -- and only the sharded one moves rows per step."""
    import numpy as np

    from ddl_amd.models import SharedArraySource
    from ddl_amd.permutation import EpochOrder

    n, gb = 300, 32
    data = (torch.arange(n) % 251).to(torch.uint8).view(n, 1, 1, 1).expand(n, 3, 8, 8).contiguous()
    src = SharedArraySource.create(f"ddl_amd_resgpu_{np.random.randint(1 << 30)}", data)
    try:
        res = run_ranks(_resident_rank_gpu, 2, src.name, n, gb, replicate, scatter, timeout=180, env=GPU_GLOO)
    finally:
        src.close()
    order = EpochOrder(n, gb, 4)
    ref = (order.perm(0).full()[: order.batches_per_epoch * gb] % 251).reshape(-1, gb)
    merged = np.concatenate([r[0] for r in res], axis=1)
    assert np.array_equal(merged, ref)
    moved_steps = sum(r[1] for r in res)
    assert (moved_steps == 0) == replicate
    assert (sum(r[2] for r in res) > 0) == replicate
