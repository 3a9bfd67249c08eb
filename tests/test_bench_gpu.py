"""bench.py on one MI355X: the driver's N=1 line produces the credited JSON with every phase's fields."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(200)
def test_bench_n1_reports_pressure_idle():
    """Phase 3 puts the loader-pressure idle into the credited line: a calibrated step at 0.9x the feed,
    its achieved ratio, and the idle % behind it next to the PatchMLP figure."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DDL_BACKEND", "MASTER_PORT")}
    env["PYTHONPATH"] = REPO
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "5",
                        "--order", "window"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["value"] > 0 and out["dtype"] == "bf16"
    p = out["pressure"]
    assert p and "error" not in p, p
    assert out["gpu_idle_pct_r090"] == p["gpu_idle_pct"] is not None
    assert 0.7 < p["ratio_measured"] < 1.1, p  # the step landed near the target ratio
    assert 0.0 <= p["gpu_idle_pct"] < 20.0
    assert out["gpu_idle_pct"] is not None  # the PatchMLP phase still runs


@pytest.mark.timeout(200)
def test_bench_one_rank_rccl_prints_dist_block():
    """A 1-rank RCCL group (DDL_BACKEND=nccl) runs the exchange and prints the self-verifying dist block:
    backend nccl, group size 1, the RCCL version, this GPU's PCI bus ID, and a device-timed all-to-all."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "DDL_REHEARSAL")}
    env.update(PYTHONPATH=REPO, DDL_BACKEND="nccl")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "5",
                        "--order", "window", "--exchange", "0.5", "--pressure-ratio", "0", "--idle-steps", "0"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    d = out["dist"]
    assert d["backend"] == "nccl" and d["group_size"] == 1 and d["rccl_version"]
    (me,) = d["ranks"]
    assert me["device_index"] == 0 and me["pci_bus_id"] and me["uuid"] is not None
    a = me["alltoall"]
    assert a["device_timed"] and a["data_ok"] and a["ms_median"] > 0 and a["alg_gbps"] > 0
    pr = out["per_rank"][0]
    assert pr["exchange_calls"] > 0 and pr["exchange_issue_wait_timed"]["exchange_issue_wait_n"] > 0
