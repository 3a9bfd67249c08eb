"""Cross-cutting utilities: logging, hook dispatch, tracing, fault injection."""

from .callbacks import execute_callbacks
from .logging import configure as configure_logging
from .logging import for_all_methods, logger, with_logging
from .tracing import ComputeIdleMeter, LoaderMetrics, trace_range

__all__ = [
    "execute_callbacks",
    "configure_logging",
    "for_all_methods",
    "logger",
    "with_logging",
    "ComputeIdleMeter",
    "LoaderMetrics",
    "trace_range",
]
