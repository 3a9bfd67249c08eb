"""Per-call debug tracing with a rank prefix (reference ddl/utils.py:25-57).

The reference's ``with_logging`` builds ``repr()`` of every argument eagerly on
every decorated call, even with DEBUG off -- including the per-batch ``mark``
(reference ddl/utils.py:28-30). Here formatting happens only when the logger
is enabled for DEBUG, so decorated hot paths cost one ``isEnabledFor`` check.
"""

from __future__ import annotations

import functools
import logging
import os
import threading
from typing import Any, Callable, TypeVar

F = TypeVar("F", bound=Callable[..., Any])

logger = logging.getLogger("ddl_amd")

_ROLE = threading.local()


def set_role(role: str, index: int = 0) -> None:
    """Record the calling thread's role (consumer / producer k) for log prefixes."""
    _ROLE.role = role
    _ROLE.index = index


def rank_prefix() -> str:
    rank = int(os.environ.get("RANK", os.environ.get("SLURM_PROCID", "0")) or 0)
    if getattr(_ROLE, "role", "consumer") == "producer":
        return f"[{rank:03d}.p{_ROLE.index}]"
    return f"[{rank:03d}]"


def _short_repr(v: Any, limit: int = 120) -> str:
    try:
        r = repr(v)
    except Exception:  # pragma: no cover - defensive
        r = f"<{type(v).__name__}>"
    return r if len(r) <= limit else r[: limit - 3] + "..."


def with_logging(func: F) -> F:
    """Log entry/exit (DEBUG) and exceptions (ERROR) of ``func``; lazy formatting."""

    @functools.wraps(func)
    def wrapper(*args: Any, **kwargs: Any) -> Any:
        if not logger.isEnabledFor(logging.DEBUG):
            try:
                return func(*args, **kwargs)
            except Exception:
                logger.exception("%s exception raised in %s", rank_prefix(), func.__qualname__)
                raise
        sig = ", ".join([_short_repr(a) for a in args] + [f"{k}={_short_repr(v)}" for k, v in kwargs.items()])
        logger.debug("%s --> %s(%s)", rank_prefix(), func.__qualname__, sig)
        try:
            result = func(*args, **kwargs)
        except Exception:
            logger.exception("%s exception raised in %s", rank_prefix(), func.__qualname__)
            raise
        logger.debug("%s <-- %s: %s", rank_prefix(), func.__qualname__, _short_repr(result))
        return result

    wrapper.__wrapped_by_ddl_logging__ = True  # type: ignore[attr-defined]
    return wrapper  # type: ignore[return-value]


def for_all_methods(decorator: Callable[[Any], Any], exclude: str | list[str] | None = None):
    """Class decorator applying ``decorator`` to every plain method in the class dict.

    Unlike the reference (which double-wraps already decorated methods, reference
    ddl/connection.py:65) a method already wrapped by ``with_logging`` is skipped;
    static/class methods and properties are left alone.
    """
    if exclude is None:
        excl: list[str] = []
    elif isinstance(exclude, str):
        excl = [exclude]
    else:
        excl = list(exclude)

    def decorate(cls):
        for name, attr in list(cls.__dict__.items()):
            if name in excl or isinstance(attr, (staticmethod, classmethod, property)):
                continue
            if callable(attr) and not getattr(attr, "__wrapped_by_ddl_logging__", False):
                setattr(cls, name, decorator(attr))
        return cls

    return decorate


def configure(level: int | str | None = None) -> None:
    """Configure the ``ddl_amd`` logger from ``level`` or ``DDL_LOG_LEVEL``."""
    lvl = level if level is not None else os.environ.get("DDL_LOG_LEVEL")
    if lvl is None:
        return
    if isinstance(lvl, str):
        lvl = getattr(logging, lvl.upper(), logging.INFO)
    logger.setLevel(lvl)
    if not logger.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(message)s"))
        logger.addHandler(h)
