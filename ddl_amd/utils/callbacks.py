"""Ordered hook dispatch (reference ddl/utils.py:9-22).

The reference's ``execute_callbacks`` returns from inside its loop, so only
``callbacks[0]`` ever runs and the appended ``GlobalShuffler`` is never
invoked (verified). Here every registered callback that
defines the hook runs, in registration order. The return value is the first
non-``None`` result (which preserves the reference's use of ``on_init``'s
return value from the user producer registered first).
"""

from __future__ import annotations

import logging
from typing import Any, Iterable

from .logging import logger, rank_prefix


def execute_callbacks(position: str, callbacks: Iterable[Any], **kwargs: Any) -> Any:
    result = None
    for cb in callbacks:
        method = getattr(cb, position, None)
        if method is None or not callable(method):
            continue
        if logger.isEnabledFor(logging.DEBUG):
            logger.debug("%s --> '%s' callback '%s'", rank_prefix(), position, type(cb).__name__)
        ret = method(**kwargs)
        if logger.isEnabledFor(logging.DEBUG):
            logger.debug("%s <-- '%s' callback '%s'", rank_prefix(), position, type(cb).__name__)
        if result is None and ret is not None:
            result = ret
    return result
