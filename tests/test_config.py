"""Every environment knob (docs/CONFIG.md) is documented, the set stays small, and each one has a test.

Knobs covered elsewhere: DDL_BACKEND (test_multirank_*), DDL_DEVICE (everywhere), DDL_PRODUCERS_PER_RANK
(test_utils), DDL_PRODUCER_MODE / DDL_FAULT_PRODUCER (test_loader_cpu), DDL_HOSTNAME (test_multirank_cpu),
DDL_FAULT_RANK (test_job_abort), DDL_REHEARSAL (test_examples, test_multirank_gpu), DDL_NATIVE_PIN
(test_stale_build). The rest are tested here.
"""

import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
MAX_KNOBS = 20


def _source_knobs() -> set[str]:
    found = set()
    files = [*ROOT.joinpath("ddl_amd").rglob("*.py"), *ROOT.joinpath("csrc").rglob("*.cpp"),
             *ROOT.joinpath("csrc").rglob("*.h"), *ROOT.joinpath("csrc").rglob("*.hip"), ROOT / "bench.py"]
    macros = set()
    for f in files:
        text = f.read_text()
        found |= set(re.findall(r"\bDDL_[A-Z][A-Z0-9_]*\b", text))
        macros |= set(re.findall(r"#define\s+(DDL_[A-Z0-9_]+)", text))
    return found - macros  # C macros (DDL_HD, DDL_SPLIT, ...) are not environment variables


def _documented_knobs() -> set[str]:
    rows = [ln for ln in (ROOT / "docs" / "CONFIG.md").read_text().splitlines() if ln.startswith("| `")]
    return {k for ln in rows for k in re.findall(r"`(DDL_[A-Z0-9_]+)`", ln.split("|")[1])}


def test_every_knob_documented_and_few():
    src, doc = _source_knobs(), _documented_knobs()
    assert src <= doc, f"undocumented: {sorted(src - doc)}"
    assert doc <= src, f"documented but gone: {sorted(doc - src)}"
    assert len(src) <= MAX_KNOBS, sorted(src)


def _py(code: str, **env) -> str:
    e = dict(os.environ, PYTHONPATH=str(ROOT), **env)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip()


def test_timeout_knob():
    assert _py("from ddl_amd.connection import DEFAULT_TIMEOUT_S as t; print(t)", DDL_TIMEOUT_S="12.5") == "12.5"


def test_trace_collectives_knob():
    assert _py("from ddl_amd.parallel.order import LEDGER; print(LEDGER.enabled)", DDL_TRACE_COLLECTIVES="1") == "True"
    assert _py("from ddl_amd.parallel.order import LEDGER; print(LEDGER.enabled)", DDL_TRACE_COLLECTIVES="0") == "False"


def test_log_level_knob():
    code = "from ddl_amd.utils.logging import configure, logger; configure(); print(logger.level)"
    assert _py(code, DDL_LOG_LEVEL="DEBUG") == "10"


def test_roctx_knob():
    code = "import ddl_amd.utils.tracing as t; print(t._ROCTX_ENABLED, t._roctx())"
    assert _py(code, DDL_ROCTX="0") == "False ()"
    assert _py("import ddl_amd.engine_dispatch as d; print(d._TRACE_ENGINE)", DDL_ROCTX="2") == "True"


def test_numa_bind_and_cpu_partition_knobs(monkeypatch):
    from ddl_amd.utils import numa

    monkeypatch.setenv("DDL_NUMA_BIND", "0")
    before = os.sched_getaffinity(0)
    assert numa.bind_to_gpu_numa(0, 1) is None and os.sched_getaffinity(0) == before
    monkeypatch.setenv("DDL_CPU_PARTITION", "0")
    assert numa.partition_after_spawn([os.getpid()], 1) is None


def test_no_autobuild_knob(monkeypatch):
    import ddl_amd._native as nat
    from ddl_amd.exceptions import NativeExtensionError

    monkeypatch.setenv("DDL_AMD_NO_AUTOBUILD", "1")
    with pytest.raises(NativeExtensionError, match="not built"):
        nat._load("_ddl_does_not_exist", "runtime")


def test_stream_stores_knob():
    code = "from ddl_amd import _native; print(_native.runtime().stream_stores())"
    assert _py(code, DDL_STREAM_STORES="0") == "False"
    assert _py(code, DDL_STREAM_STORES="1") == "True"


def test_stream_store_copies_are_exact():
    """Every host window copy gives the same bytes with and without streaming stores, for unaligned
    destinations and lengths around the 1 KiB switch and the 16 / 64-byte store blocks."""
    import numpy as np

    from ddl_amd import _native

    rt = _native.runtime()
    rng = np.random.default_rng(0)
    src = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    try:
        for nt in (True, False):
            rt.set_stream_stores(nt)
            for row in (1, 17, 1023, 1024, 1025, 4099, 65536 + 48):
                n = min(64, src.size // row)
                idx = rng.permutation(n).astype(np.int64)
                dst = np.zeros(n * row + 3, dtype=np.uint8)
                rt.gather_rows(dst.ctypes.data + 3, src.ctypes.data, row, idx, n, 4)
                want = src[: n * row].reshape(n, row)[idx].reshape(-1)
                assert np.array_equal(dst[3:], want), (nt, row)
            dst = np.zeros(src.size + 5, dtype=np.uint8)
            rt.parallel_copy(dst.ctypes.data + 5, src.ctypes.data, src.size, 3)
            assert np.array_equal(dst[5:], src)
    finally:
        rt.set_stream_stores(True)


def test_verify_order_knob(monkeypatch):
    """DDL_VERIFY_ORDER=1 turns on the per-window order check of indexed loaders by default."""
    import numpy as np
    import torch

    import ddl_amd
    from ddl_amd.models import IndexedProducer, SharedArraySource

    monkeypatch.setenv("DDL_DEVICE", "cpu")
    monkeypatch.setenv("DDL_VERIFY_ORDER", "1")
    n, gb = 256, 32
    src = SharedArraySource.create(f"ddl_amd_cfg_{np.random.randint(1 << 30)}", torch.arange(2 * n).view(n, 2))
    try:
        with ddl_amd.start(n_producers=1) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, gb), gb, conn, 1, env=env, auto_mark=True,
                                               order=ddl_amd.OrderSpec(mode="indexed", seed=3))
            assert dl._verify is not None
            assert sum(1 for _ in dl) == n // gb
            assert dl.verified_windows == n // gb
            dl.close()
    finally:
        src.close()
