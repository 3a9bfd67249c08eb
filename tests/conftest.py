import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault("PYTHONPATH", REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _no_shm_leak():
    if os.environ.get("PYTEST_XDIST_WORKER"):  # parallel workers see each other's live segments
        yield
        return
    before = set(os.listdir("/dev/shm"))
    yield
    leaked = [f for f in set(os.listdir("/dev/shm")) - before if f.startswith("ddl_amd")]
    assert not leaked, f"leaked shm segments: {leaked}"
