"""Host C++ runtime under sanitizers (SURVEY §5 "Race detection"): ASAN+UBSAN and TSAN
builds of csrc/runtime/tests/stress.cpp (producer/consumer threads over two mappings of
one arena, shutdown while blocked, concurrent host gather pool). Host code only."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(REPO, "csrc", "runtime", "arena.cpp"), os.path.join(REPO, "csrc", "runtime", "tests", "stress.cpp")]


def _build(tmp_path, flags, name):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", *flags, *SRC, "-o", exe, "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        if "sanitizer" in r.stderr or "cannot find" in r.stderr:
            pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
        raise AssertionError(r.stderr)
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("kind,flags", [
    ("asan_ubsan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"]),
    ("tsan", ["-fsanitize=thread"]),
])
def test_runtime_stress_under_sanitizer(tmp_path, kind, flags):
    exe = _build(tmp_path, flags, f"stress_{kind}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "stress ok" in r.stdout
