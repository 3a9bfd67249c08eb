"""The auto copy policy's trigger (csrc/kernels/copy_mode.h), built with g++ and run on the CPU: stays
alternating when loader-bound, switches to one stream after 3 copies that waited for their ring buffer,
ignores an isolated wait, and switches back after 6 back-to-back copies."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_copy_mode_trigger(tmp_path):
    exe = str(tmp_path / "copy_mode_test")
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(REPO, "csrc", "kernels"),
                    os.path.join(REPO, "csrc", "kernels", "tests", "copy_mode_test.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "copy_mode ok" in r.stdout, r.stdout + r.stderr
