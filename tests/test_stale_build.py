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
