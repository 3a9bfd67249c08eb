"""In-tree native build for ddl_amd (no setuptools / hipify involved).

Two shared objects are produced next to this file:

* ``_ddl_runtime``  -- host C++ runtime (shm arena, futex hand-off, host
  gather pool). Built with g++; no torch / HIP dependency so producer worker
  processes and CPU-only hosts can load it.
* ``_ddl_hip``      -- hand-written CDNA4 (gfx950) HIP kernels + torch
  bindings. Kernels are compiled with ``hipcc --offload-arch=gfx950``; the
  module links against the HIP runtime bundled in torch/lib so a single HIP
  runtime lives in the process.

Each shared object embeds a SHA-256 of its source inputs (``source_hash``; the marker
``ddl-source-hash=<hex>`` in a generated translation unit). ``_native`` compares it with the tree
before importing, so an edit under ``csrc/`` without a rebuild is rebuilt (or, with
``DDL_AMD_NO_AUTOBUILD=1``, reported) instead of silently running the old binary.

Usage: ``python -m ddl_amd._build [--only runtime|hip] [--force] [-j N]``.
"""

from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = "gfx950"  # MI355X (CDNA4) only
VERBOSE = False  # echo the compiler output (``--verbose``)


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def _py_includes() -> list[str]:
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _torch_paths() -> tuple[str, list[str]]:
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return os.path.join(root, "lib"), inc


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout)
        raise RuntimeError(f"native build failed ({proc.returncode}): {' '.join(cmd[:4])} ...")
    if VERBOSE:
        sys.stderr.write(proc.stdout)


HASH_MARKER = b"ddl-source-hash="


def runtime_inputs() -> list[str]:
    srcs = [os.path.join(CSRC, "runtime", f) for f in ("arena.cpp", "fileio.cpp", "numa.cpp", "bindings.cpp")]
    return srcs + [os.path.join(CSRC, "runtime", h) for h in ("arena.h", "feistel.h", "fileio.h", "numa.h")]


def hip_inputs() -> list[str]:
    """Every file compiled into ``_ddl_hip``: the kernels, the host C++ (stager, engine, bindings, the
    arena), and the headers they include."""
    return sorted(_kernel_sources() + glob.glob(os.path.join(CSRC, "kernels", "*.h")) +
                  [os.path.join(CSRC, "kernels", f) for f in ("bindings.cpp", "stager.cpp", "engine.cpp")] +
                  [os.path.join(CSRC, "runtime", f) for f in ("arena.cpp", "arena.h", "feistel.h")])


def sources_present() -> bool:
    """The csrc tree is here (an installed package without it cannot be checked)."""
    return os.path.isdir(os.path.join(CSRC, "runtime")) and os.path.isdir(os.path.join(CSRC, "kernels"))


def source_hash(paths: list[str]) -> str:
    """SHA-256 over the inputs' paths (relative to csrc/) and contents, and the target architecture."""
    h = hashlib.sha256(ARCH.encode())
    for p in sorted(paths):
        h.update(os.path.relpath(p, CSRC).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def embedded_hash(target: str) -> str | None:
    """The source hash a built shared object carries, or None (missing file, or built without one)."""
    try:
        with open(target, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(HASH_MARKER)
    if i < 0:
        return None
    h = data[i + len(HASH_MARKER):i + len(HASH_MARKER) + 64]
    return h.decode() if len(h) == 64 else None


def is_stale(which: str) -> bool:
    """``which`` ("runtime" / "hip") is missing, or was built from other sources than the tree's."""
    target, inputs = (runtime_target(), runtime_inputs()) if which == "runtime" else (hip_target(), hip_inputs())
    if not os.path.exists(target):
        return True
    if not sources_present():
        return False
    return embedded_hash(target) != source_hash(inputs)


def _hash_source(name: str, digest: str) -> str:
    """A translation unit that carries ``digest`` in the shared object (kept by ``used``)."""
    os.makedirs(BUILD, exist_ok=True)
    path = os.path.join(BUILD, f"{name}_source_hash.cpp")
    with open(path, "w") as f:
        f.write(f'__attribute__((used)) extern const char ddl_{name}_source_hash[] = '
                f'"{HASH_MARKER.decode()}{digest}";\n')
    return path


def runtime_target() -> str:
    return os.path.join(PKG_DIR, "_ddl_runtime" + EXT_SUFFIX)


def hip_target() -> str:
    return os.path.join(PKG_DIR, "_ddl_hip" + EXT_SUFFIX)


def build_runtime(force: bool = False, extra_flags: list[str] | None = None) -> str:
    deps = runtime_inputs()
    srcs = [d for d in deps if d.endswith(".cpp")]
    out = runtime_target()
    digest = source_hash(deps)
    if not force and not _newer(out, deps) and embedded_hash(out) == digest:
        return out
    srcs.append(_hash_source("runtime", digest))
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
    cmd += [f"-I{p}" for p in _py_includes()]
    cmd += list(extra_flags or [])
    cmd += srcs + ["-o", out + ".tmp", "-lpthread", "-lrt"]
    _run(cmd)
    os.replace(out + ".tmp", out)
    return out


def _kernel_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))


def build_hip(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    torch_lib, _ = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    out = hip_target()
    kernel_srcs = _kernel_sources()
    binding = os.path.join(CSRC, "kernels", "bindings.cpp")
    # host-only C++ compiled into the HIP module: the native stager and its own copy
    # of the arena implementation (it drives the consumer's Arena object by address)
    host_srcs = [os.path.join(CSRC, "kernels", "stager.cpp"), os.path.join(CSRC, "kernels", "engine.cpp"),
                 os.path.join(CSRC, "runtime", "arena.cpp")]
    headers = headers + [os.path.join(CSRC, "runtime", "arena.h")]

    jobs_list: list[tuple[list[str], str]] = []
    objs: list[str] = []
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{os.path.join(CSRC, 'runtime')}", f"-I{os.path.join(CSRC, 'kernels')}"]
    for src in kernel_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            cmd = [hipcc, f"--offload-arch={ARCH}", "-c", src, "-o", obj, "-munsafe-fp-atomics"] + common
            jobs_list.append((cmd, obj))
    for src in host_srcs:
        obj = os.path.join(BUILD, "hip_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append(([hipcc, "-c", src, "-o", obj, "-fvisibility=hidden"] + common, obj))
    bobj = os.path.join(BUILD, "bindings.cpp.o")
    objs.append(bobj)
    if force or _newer(bobj, [binding] + headers):
        cmd = [hipcc, "-c", binding, "-o", bobj] + common
        cmd += [f"-I{p}" for p in _py_includes()] + ["-fvisibility=hidden"]
        jobs_list.append((cmd, bobj))
    digest = source_hash(hip_inputs())
    stale = embedded_hash(out) != digest
    if force or stale or jobs_list:
        hobj = os.path.join(BUILD, "hip_source_hash.o")
        jobs_list.append(([hipcc, "-c", _hash_source("hip", digest), "-o", hobj, "-fPIC"], hobj))
    objs.append(os.path.join(BUILD, "hip_source_hash.o"))

    if jobs_list:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(lambda j: _run(j[0]), jobs_list))
    if force or jobs_list or stale or _newer(out, objs):
        cmd = [hipcc, "-shared", "-fPIC", *objs, "-o", out + ".tmp", f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}",
               "-l:libamdhip64.so", "-l:libhsa-runtime64.so", "-lpthread", "-lrt"]
        _run(cmd)
        os.replace(out + ".tmp", out)
    return out


def build_benchmarks(force: bool = False) -> list[str]:
    """Standalone gfx950 microbenchmarks (``benchmarks/*.hip`` -> ``benchmarks/bin/``): HIP executables that
    need no torch, built next to the extensions so the GPU box runs them without compiling."""
    out = []
    bin_dir = os.path.join(REPO, "benchmarks", "bin")
    os.makedirs(bin_dir, exist_ok=True)
    for src in sorted(glob.glob(os.path.join(REPO, "benchmarks", "*.hip"))):
        target = os.path.join(bin_dir, os.path.splitext(os.path.basename(src))[0])
        deps = [src, *glob.glob(os.path.join(CSRC, "kernels", "*.h"))]
        if force or _newer(target, deps):
            _run([_hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-I", os.path.join(CSRC, "kernels"),
                  src, "-o", target, "-lhsa-runtime64"])
        out.append(target)
    return out


def build_all(force: bool = False, jobs: int = 8) -> None:
    build_runtime(force=force)
    build_hip(force=force, jobs=jobs)
    build_benchmarks(force=force)


def main(argv: list[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--only", choices=["runtime", "hip", "benchmarks"], default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    ap.add_argument("-v", "--verbose", action="store_true", help="echo the compiler output")
    a = ap.parse_args(argv)
    global VERBOSE
    VERBOSE = a.verbose
    if a.only in (None, "runtime"):
        print(build_runtime(force=a.force))
    if a.only in (None, "hip"):
        print(build_hip(force=a.force, jobs=a.jobs))
    if a.only in (None, "benchmarks"):
        print("\n".join(build_benchmarks(force=a.force)))


if __name__ == "__main__":
    main()
