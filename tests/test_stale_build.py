"""Stale-binary guard (``ddl_amd/_build.py`` source hash, ``ddl_amd/_native._check_fresh``).

The reference has no native code; this protects the pipeline that ships in-tree ``.so`` files to the GPU
box: an edit under ``csrc/`` without a rebuild must never run the old binary silently. A copy of the
package and its ``csrc/`` tree is edited, then loaded in a fresh interpreter.
"""

import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LOAD = "import ddl_amd._native as n, ddl_amd._build as b; n.runtime(); print('STALE', b.is_stale('runtime'))"


def _copy_tree(tmp_path):
    root = tmp_path / "repo"
    shutil.copytree(os.path.join(REPO, "ddl_amd"), root / "ddl_amd",
                    ignore=shutil.ignore_patterns("__pycache__", "_ddl_hip*.so"))
    shutil.copytree(os.path.join(REPO, "csrc"), root / "csrc", ignore=shutil.ignore_patterns("tests"))
    return root


def _run(root, **env):
    e = {k: v for k, v in os.environ.items() if k != "DDL_AMD_NO_AUTOBUILD"}
    e.update(PYTHONPATH=str(root), **env)
    return subprocess.run([sys.executable, "-c", LOAD], cwd=str(root), env=e, capture_output=True, text=True,
                          timeout=600)


def test_source_hash_is_embedded_and_matches_the_tree():
    from ddl_amd import _build

    assert _build.embedded_hash(_build.runtime_target()) == _build.source_hash(_build.runtime_inputs())
    assert not _build.is_stale("runtime")


@pytest.mark.timeout(900)
def test_edited_csrc_is_reported_or_rebuilt(tmp_path):
    root = _copy_tree(tmp_path)
    ok = _run(root, DDL_AMD_NO_AUTOBUILD="1")
    assert ok.returncode == 0 and "STALE False" in ok.stdout, ok.stderr[-2000:]
    # an edit of a runtime source without a rebuild
    src = root / "csrc" / "runtime" / "arena.cpp"
    src.write_text(src.read_text() + "\n// edited after the build\n")
    so = next((root / "ddl_amd").glob("_ddl_runtime*.so"))
    before = so.read_bytes()
    refused = _run(root, DDL_AMD_NO_AUTOBUILD="1")
    assert refused.returncode != 0 and "stale" in refused.stderr, refused.stderr[-2000:]
    assert so.read_bytes() == before  # nothing was loaded or rebuilt
    rebuilt = _run(root)
    assert rebuilt.returncode == 0 and "STALE False" in rebuilt.stdout, rebuilt.stderr[-2000:]
    assert so.read_bytes() != before


def test_children_load_the_parents_build_or_refuse(tmp_path):
    """A producer spawned mid-job loads exactly the binary its consumer loaded (DDL_NATIVE_PIN, inherited): it
    never rebuilds a stale one under a live job, and a file that changed under the job is an error -- the
    consumer and its producers never run different builds over one arena."""
    root = _copy_tree(tmp_path)
    first = _run(root, DDL_AMD_NO_AUTOBUILD="1")
    assert first.returncode == 0 and "STALE False" in first.stdout, first.stderr[-2000:]
    so = next((root / "ddl_amd").glob("_ddl_runtime*.so"))
    code = "import os, ddl_amd._native as n; n.runtime(); print(os.environ['DDL_NATIVE_PIN'])"
    e = {k: v for k, v in os.environ.items() if k not in ("DDL_AMD_NO_AUTOBUILD", "DDL_NATIVE_PIN")}
    r = subprocess.run([sys.executable, "-c", code], cwd=str(root), env=dict(e, PYTHONPATH=str(root)),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    pin = r.stdout.strip().splitlines()[-1]
    assert str(so.resolve()) in pin
    # csrc/ edited after the consumer loaded its build: a child with the pin loads that build, no rebuild
    src = root / "csrc" / "runtime" / "arena.cpp"
    src.write_text(src.read_text() + "\n// edited mid-job\n")
    before = so.read_bytes()
    child = _run(root, DDL_NATIVE_PIN=pin)
    assert child.returncode == 0 and "STALE True" in child.stdout, child.stderr[-2000:]
    assert so.read_bytes() == before
    # the .so itself replaced under the job (a rebuild by someone else): the child refuses
    digest = pin.rpartition("=")[2]
    bad = _run(root, DDL_NATIVE_PIN=f"{so.resolve()}={'0' * len(digest)}")
    assert bad.returncode != 0 and "changed under the running job" in bad.stderr, bad.stderr[-2000:]
