"""Real multi-GPU RCCL runs (2..8 MI355X of one node): the driver's N > 1 line and the replicated resident
layout over xGMI. gpurun boxes expose one GPU, so these tests are skipped there; on a multi-GPU node they are
the checks the one-card gloo rehearsals (``test_multirank_gpu.py``) stand in for. RCCL refuses two ranks on one
GPU, so every rank here gets its own device (``LOCAL_RANK`` -> ``cuda:LOCAL_RANK``).
"""

import json
import os
import subprocess
import sys

import pytest
import torch

from tests.mp_harness import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_GPUS = min(torch.cuda.device_count(), 8)  # counting devices does not initialise HIP

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(N_GPUS < 2, reason="needs >= 2 GPUs on this node (RCCL)")]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("DDL_REHEARSAL", "DDL_BACKEND", "DDL_DEVICE",
                                                            "WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = REPO
    return env


def _torchrun(n, script, *args, timeout=280):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, script), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])


@pytest.mark.timeout(300)
def test_bench_line_verifies_rccl_over_distinct_gpus():
    """The driver's command at N = all GPUs of the node: RCCL over N distinct PCI bus IDs, a device-timed
    all-to-all on the DP group, one collective order, and every rank fed."""
    out = _torchrun(N_GPUS, "bench.py", "--gpus", str(N_GPUS), "--steps", "20", "--warmup", "5",
                    "--order", "window", "--pressure-ratio", "0")
    d = out["dist"]
    assert d["backend"] == "nccl" and d["group_size"] == N_GPUS and d["verified"] is True and not d["problems"]
    assert d["distinct_gpus"] == N_GPUS and len({r["pci_bus_id"] for r in d["ranks"]}) == N_GPUS
    assert all(r["alltoall"]["data_ok"] and r["alltoall"]["device_timed"] for r in d["ranks"])
    order = out["collective_order"]
    assert order["same_order"] is True and order["groups"] == 1
    assert out["n_gpus"] == N_GPUS and out["value"] > 0
    assert all(r["h2d_bytes_timed"] > 0 and r["exchange_calls"] > 0 for r in out["per_rank"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("replicate", ["true", "false"])
def test_resident_layouts_over_rccl(replicate):
    """Config 5 over RCCL: the replicated layout moves nothing per step, the sharded one all-to-alls."""
    out = _torchrun(N_GPUS, os.path.join("benchmarks", "bench_resident.py"), "--steps", "50", "--warmup", "10",
                    "--depths", "2", "--n-samples", str(1024 * N_GPUS), "--replicate", replicate)
    (res,) = out["sweep"]
    assert out["dist"]["verified"] is True and res["samples_per_s"] > 0
    assert res["mode"] == ("replicated" if replicate == "true" else "sharded")
    assert (res["xgmi_GB_sent_per_rank_steps"] == 0) == (replicate == "true")
