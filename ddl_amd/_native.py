"""Loading of the in-tree native extensions.

``runtime()`` returns the host C++ runtime (always required: producers and the
consumer hand slots over through it). ``hip()`` returns the gfx950 kernel
module. On a GPU host a missing/broken HIP extension is an error, never a
silent fallback to eager PyTorch: ``hip()`` raises ``NativeExtensionError``.
If an extension is missing it is built in-tree once (under a file lock, so
concurrently starting producer processes do not race); set
``DDL_AMD_NO_AUTOBUILD=1`` to disable.
"""

from __future__ import annotations

import fcntl
import importlib
import os
import threading
from types import ModuleType

from .exceptions import NativeExtensionError

_lock = threading.Lock()
_cache: dict[str, ModuleType] = {}


def _build_locked(which: str) -> None:
    from . import _build

    os.makedirs(_build.BUILD, exist_ok=True)
    with open(os.path.join(_build.BUILD, ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if which == "runtime":
                _build.build_runtime()
            else:
                _build.build_hip()
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _load(name: str, which: str) -> ModuleType:
    with _lock:
        if name in _cache:
            return _cache[name]
        try:
            mod = importlib.import_module(f"ddl_amd.{name}")
        except ImportError as first:
            if os.environ.get("DDL_AMD_NO_AUTOBUILD"):
                raise NativeExtensionError(f"ddl_amd.{name} is not built ({first}); run `python -m ddl_amd._build`")
            try:
                _build_locked(which)
                mod = importlib.import_module(f"ddl_amd.{name}")
            except Exception as e:  # pragma: no cover - depends on toolchain
                raise NativeExtensionError(f"ddl_amd.{name} failed to build/load: {e}") from e
        _cache[name] = mod
        return mod


def runtime() -> ModuleType:
    return _load("_ddl_runtime", "runtime")


def hip() -> ModuleType:
    import torch  # noqa: F401  (torch's HIP runtime must be the one in the process)

    return _load("_ddl_hip", "hip")


def gpu_available() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_available())
    except Exception:  # pragma: no cover
        return False
