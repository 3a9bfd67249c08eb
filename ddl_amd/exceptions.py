"""Typed errors of the loader.

The reference has a single ``DoesNotMatchError`` whose constructor is misspelt
``__init`` (reference ddl/exceptions.py:1-5), so it behaves as a plain
``Exception(value, message)``. Here the constructor works and every failure
mode the reference leaves as a hang or a bare ``SystemExit``/``Abort`` has its
own type.
"""

from __future__ import annotations

from typing import Any


class DDLError(RuntimeError):
    """Base class of every ddl_amd error."""


class DoesNotMatchError(DDLError):
    """A value does not match what the topology/metadata requires.

    Mirrors reference ddl/exceptions.py (with a working ``__init__``).
    """

    def __init__(self, value: Any, message: str):
        self.value = value
        self.message = message
        super().__init__(message)


class TopologyError(DoesNotMatchError):
    """Rank layout is invalid (e.g. a GPU group spanning nodes, bad sizes)."""


class ShapeMismatchError(DoesNotMatchError):
    """Producer metadata disagree (shape, splits, dtype, batches per window)."""


class CommunicatorMismatchError(DoesNotMatchError):
    """A loader collective was about to be issued on a process group other than the DP group
    (``env.process_group``): it would run on another communicator / stream than DDP's and could
    deadlock against it across ranks (``parallel/order.py``)."""


class DDLTimeoutError(DDLError, TimeoutError):
    """A bounded wait expired (producer never published / consumer never released)."""


class PeerDeathError(DDLError):
    """A peer process died (or reported failure) while we were waiting on it."""

    def __init__(self, message: str, producer_index: int | None = None, pid: int | None = None):
        self.producer_index = producer_index
        self.pid = pid
        super().__init__(message)


class DataIntegrityError(DDLError):
    """A delivered window is not the one the epoch order says comes next (``verify_order``): a
    producer/consumer cursor disagreement, a stale or reused slot, or a bad resume."""


class ShutdownError(DDLError):
    """The loader was shut down while an operation was waiting."""


class NativeExtensionError(DDLError, ImportError):
    """A native (C++/HIP) extension is missing or failed to load."""
