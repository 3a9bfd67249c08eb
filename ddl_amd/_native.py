"""Loading of the in-tree native extensions.

``runtime()`` returns the host C++ runtime (always required: producers and the
consumer hand slots over through it). ``hip()`` returns the gfx950 kernel
module. On a GPU host a missing/broken HIP extension is an error, never a
silent fallback to eager PyTorch: ``hip()`` raises ``NativeExtensionError``.
If an extension is missing, or STALE -- the source hash it embeds differs from
the ``csrc/`` tree's (``_build.is_stale``) -- it is (re)built in-tree before the
import (under a file lock, so concurrently starting producer processes do not
race); with ``DDL_AMD_NO_AUTOBUILD=1`` either case raises instead.

A process that has loaded an extension pins it for its children: ``DDL_NATIVE_PIN`` (set here, inherited
by every producer or helper process spawned later) names each loaded ``.so`` and the source hash it
carries. A child loading the same file never rebuilds it -- it loads exactly that binary, or raises
``NativeExtensionError`` when the file changed under the job (``csrc/`` edited and rebuilt mid-run), so a
consumer and its producers never run different builds over one shared arena.
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


def _check_fresh(name: str, which: str) -> None:
    """Rebuild a stale extension before it is imported (a loaded module cannot be replaced), or raise with
    ``DDL_AMD_NO_AUTOBUILD``. A missing one is left to the import below."""
    from . import _build

    target = _build.runtime_target() if which == "runtime" else _build.hip_target()
    if not os.path.exists(target) or not _build.is_stale(which):
        return
    if os.environ.get("DDL_AMD_NO_AUTOBUILD"):
        raise NativeExtensionError(
            f"ddl_amd.{name} is stale: built from other sources than csrc/ holds; run `python -m ddl_amd._build`")
    try:
        _build_locked(which)
    except Exception as e:  # pragma: no cover - depends on toolchain
        raise NativeExtensionError(f"ddl_amd.{name} is stale and failed to rebuild: {e}") from e


_PIN_ENV = "DDL_NATIVE_PIN"


def _pins() -> dict[str, str]:
    """``{realpath of a loaded .so: its source hash}`` pinned by an ancestor process."""
    out = {}
    for item in filter(None, os.environ.get(_PIN_ENV, "").split(";")):
        path, _, digest = item.rpartition("=")
        if path:
            out[path] = digest
    return out


def _pin(path: str) -> None:
    from . import _build

    digest = _build.embedded_hash(path)
    if digest is None:
        return
    pins = _pins()
    pins[os.path.realpath(path)] = digest
    os.environ[_PIN_ENV] = ";".join(f"{p}={d}" for p, d in pins.items())


def _check_pinned(name: str, which: str) -> bool:
    """True when an ancestor pinned this extension's file: it is loaded as is (no staleness check, no rebuild),
    provided it still carries the pinned hash; a file that changed under the job raises."""
    from . import _build

    target = _build.runtime_target() if which == "runtime" else _build.hip_target()
    want = _pins().get(os.path.realpath(target))
    if want is None:
        return False
    have = _build.embedded_hash(target)
    if have != want:
        raise NativeExtensionError(
            f"ddl_amd.{name} changed under the running job: the parent process loaded the build of source hash "
            f"{want[:12]}, the file now holds {str(have)[:12]} (rebuilt mid-run?); restart the job")
    return True


def _load(name: str, which: str) -> ModuleType:
    with _lock:
        if name in _cache:
            return _cache[name]
        if not _check_pinned(name, which):
            _check_fresh(name, which)
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
        if getattr(mod, "__file__", None):
            _pin(mod.__file__)
        return mod


def runtime() -> ModuleType:
    first = "_ddl_runtime" not in _cache
    mod = _load("_ddl_runtime", "runtime")
    if first and os.environ.get("DDL_STREAM_STORES", "1") == "0":  # producer processes inherit the setting
        mod.set_stream_stores(False)
    return mod


def hip() -> ModuleType:
    import torch  # noqa: F401  (torch's HIP runtime must be the one in the process)

    return _load("_ddl_hip", "hip")


def gpu_available() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_available())
    except Exception:  # pragma: no cover
        return False
