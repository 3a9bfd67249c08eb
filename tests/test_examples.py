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
