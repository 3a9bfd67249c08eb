"""The reference's only test runs its harness under ``mpirun -np 4`` and checks the exit code
(reference tests/test_ddl.py:8-28). Same here for the example harness, 1 rank (1 consumer + 3
producers, the -np 4 layout) and 2 DP ranks via torchrun -- plus the output is checked."""

import os
import subprocess
import sys

import pytest

from tests.mp_harness import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(REPO, "examples", "run_ddl.py")


def _env():
    return dict(os.environ, PYTHONPATH=REPO)


@pytest.mark.timeout(200)
def test_example_single_rank():
    r = subprocess.run([sys.executable, SCRIPT, "--epochs", "3"], capture_output=True, text=True, timeout=180,
                       env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    assert "epoch 3/3: 24 batches" in r.stdout and "Training finished" in r.stdout


@pytest.mark.timeout(300)
def test_example_two_ranks_torchrun():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), SCRIPT, "--epochs", "2", "--timesteps", "4"]
    # two ranks on one box: rehearse on CPU/gloo (RCCL refuses two ranks on one GPU)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=dict(_env(), DDL_DEVICE="cpu"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "epoch 2/2: 4 batches" in r.stdout  # 4*10052/2 rows per window // 4096


@pytest.mark.timeout(300)
def test_bench_contract_two_ranks_torchrun():
    """bench.py's driver contract at N=2 (the driver's launch line), rehearsed on CPU/gloo:
    exchange 0.5 over the DP group, DDP train step, one strict-JSON line from rank 0."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "6", "--warmup", "2", "--window", "64", "--batch", "16", "--idle-steps", "3",
           "--model-dim", "64", "--model-depth", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280,
                       env=dict(_env(), DDL_DEVICE="cpu", DDL_REHEARSAL="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0], parse_constant=lambda c: pytest.fail(f"non-JSON constant {c}"))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 2 and out["steps"] == 6 and out["warmup"] == 2 and out["value"] > 0
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 32
    assert out["config"]["exchange_fraction"] == 0.5
    assert "DDP" in out["train_step"]["model"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("method,launch", [("alltoall", "torchrun"), ("sendrecv_replace", "self")])
def test_bench_eight_ranks(method, launch):
    """The driver's N=8 run rehearsed on CPU/gloo: 8 ranks x 3 producers, a window exchange every
    4 batches in both exchange methods, then 8-rank DDP. Launched by torchrun (the driver's line) and
    by ``python bench.py --gpus 8`` alone (bench.py spawns the ranks itself). Checks that every rank
    issues the loader's exchanges and the DDP all-reduces in the same order (collective ledger
    digests compared across ranks) and that the run completes (no cross-rank deadlock)."""
    import json

    args = [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "12", "--warmup", "2", "--window", "64",
            "--batch", "16", "--idle-steps", "3", "--model-dim", "64", "--model-depth", "1",
            "--exchange-method", method]
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args]
        env = dict(_env(), DDL_DEVICE="cpu", DDL_REHEARSAL="1")
    else:
        cmd = [sys.executable, *args]
        env = {k: v for k, v in _env().items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        env.update(DDL_DEVICE="cpu", DDL_REHEARSAL="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 128
    # the line says what it is: a gloo rehearsal on 8 CPU ranks, not RCCL over 8 GPUs
    d = out["dist"]
    assert d["backend"] == "gloo" and d["group_size"] == 8 and d["world_size"] == 8
    assert d["verified"] is False and d["rehearsal"] is True and d["problems"]
    assert [r_["rank"] for r_ in d["ranks"]] == list(range(8))
    assert all(r_["alltoall"]["data_ok"] and r_["alltoall"]["bytes"] > 0 for r_ in d["ranks"])
    assert out["config"]["exchange_fraction"] == 0.5 and out["value"] > 0
    order = out["collective_order"]
    assert order["same_order"] is True and order["groups"] == 1
    assert order["by_kind"]["loader.exchange"] >= 4 and order["by_kind"]["ddp.allreduce"] >= 4
    assert len(out["per_rank"]) == 8 and all(r_["exchange_calls"] >= 3 for r_ in out["per_rank"])


@pytest.mark.timeout(300)
def test_bench_refuses_unverified_eight_ranks():
    """The driver's N=8 line must prove RCCL over 8 distinct GPUs: 8 ranks that are not (here gloo on the
    CPU) exit non-zero before measuring, print no JSON line, and say why -- unless DDL_REHEARSAL=1."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "8", "--steps", "4", "--warmup", "1", "--window", "64", "--batch", "16", "--producers", "1",
           "--a2a-probe-mb", "1"]
    env = {k: v for k, v in _env().items() if k != "DDL_REHEARSAL"}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=dict(env, DDL_DEVICE="cpu"))
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "not RCCL" in r.stderr and "'gloo'" in r.stderr and '"group_size": 8' in r.stderr


def test_dist_block_single_rank_and_checks():
    """dist_block / require_verified on hand-made layouts: N=1 needs nothing; N>1 needs RCCL over N distinct
    GPUs, or the rehearsal label."""
    from ddl_amd.parallel.report import dist_block, require_verified
    from ddl_amd.types import DDLEnv

    b = dist_block(DDLEnv(rank=0, world_size=1, hostname="h", device="cpu"))
    assert b["world_size"] == 1 and b["backend"] is None and b["verified"] is None
    assert require_verified(b) is None and b["rccl_version"]
    fake = dict(b, world_size=8, verified=False, rehearsal=False, problems=["8 ranks on 1 distinct GPU(s)"])
    assert "distinct GPU" in require_verified(fake)
    assert require_verified(dict(fake, rehearsal=True)) is None
    assert require_verified(dict(fake, verified=True)) is None


@pytest.mark.timeout(60)
def test_bench_refuses_world_size_mismatch():
    """--gpus N under a launcher with a different WORLD_SIZE exits non-zero instead of running 1 rank."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, timeout=50, env=dict(_env(), WORLD_SIZE="1", RANK="0", DDL_DEVICE="cpu"))
    assert r.returncode == 2 and "refusing" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("token_dtype", ["auto", "int32"])
def test_bench_tokens_two_ranks(token_dtype):
    """BASELINE config 4's bench at 2 ranks (CPU/gloo): local rank 0 creates the corpus (uint16 on the wire
    with "auto": the synthetic vocabulary fits), the other rank attaches to it with the right id width, and
    the token count is the delivered one."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "benchmarks", "bench_tokens.py"), "--steps", "5", "--warmup", "2", "--idle-steps", "0",
           "--batch", "64", "--n-seqs", "1024", "--token-dtype", token_dtype]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=dict(_env(), DDL_DEVICE="cpu"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["token_wire_dtype"] == ("uint16" if token_dtype == "auto" else "int32")
    assert abs(out["value"] / out["value_est_from_mean_len"] - 1) < 0.2


@pytest.mark.timeout(300)
@pytest.mark.parametrize("replicate", ["true", "false"])
def test_bench_resident_two_ranks(replicate):
    """BASELINE config 5's bench at 2 ranks (CPU/gloo rehearsal): both layouts run, say which they are, and
    the replicated one moves nothing per step."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "benchmarks", "bench_resident.py"), "--steps", "6", "--warmup", "2", "--batch", "8",
           "--n-samples", "256", "--depths", "1", "--replicate", replicate]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280,
                       env=dict(_env(), DDL_DEVICE="cpu", DDL_REHEARSAL="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    (res,) = out["sweep"]
    assert out["n_gpus"] == 2 and res["samples_per_s"] > 0 and out["dist"]["rehearsal"] is True
    assert res["mode"] == ("replicated" if replicate == "true" else "sharded")
    assert (res["xgmi_GB_sent_per_rank_steps"] == 0) == (replicate == "true")


@pytest.mark.timeout(200)
def test_bench_plumbing_config1_two_ranks():
    """BASELINE config 1 (1k x 3x32x32, world 2, CPU): exactly-once delivery every epoch, one JSON line."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "benchmarks", "bench_plumbing.py"), "--epochs", "3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=dict(_env(), DDL_DEVICE="cpu"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["world_size"] == 2 and out["exactly_once_every_epoch"] is True and out["samples_per_s"] > 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("script,args", [("resident_images.py", ["--n-samples", "512", "--epochs", "2"]),
                                         ("resident_images.py", ["--n-samples", "512", "--epochs", "1",
                                                                 "--replicate", "true"]),
                                         ("tokens_packed.py", ["--n-seqs", "256", "--epochs", "2"]),
                                         ("tokens_packed.py", ["--n-seqs", "256", "--epochs", "1", "--mode", "pad"]),
                                         ("torch_dataset.py", ["--n-samples", "256", "--epochs", "2", "--batch-size", "16"])])
@pytest.mark.parametrize("ranks", [1, 2])
def test_usage_examples(script, args, ranks):
    """The usage examples run end to end on CPU, alone and as two torchrun ranks (gloo)."""
    path = os.path.join(REPO, "examples", script)
    if ranks == 1:
        cmd = [sys.executable, path, *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), path, *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=dict(_env(), DDL_DEVICE="cpu"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "epoch 0:" in r.stdout


@pytest.mark.timeout(200)
@pytest.mark.parametrize("impl", ["ddl", "torch"])
def test_bench_dataloader_cpu(impl):
    """benchmarks/bench_dataloader.py (the drop-in comparison) runs on CPU and prints one JSON line."""
    import json

    cmd = [sys.executable, os.path.join(REPO, "benchmarks", "bench_dataloader.py"), "--impl", impl,
           "--workers", "2", "--batch", "32", "--n-samples", "1024", "--steps", "4", "--warmup", "1",
           "--idle-steps", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=dict(_env(), DDL_DEVICE="cpu"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["samples_per_s"] > 0 and out["batch"] == 32 and out["workers"] == 2
