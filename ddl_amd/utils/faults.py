"""Fault injection hooks for tests (SURVEY §5 "Failure detection").

``DDL_FAULT_PRODUCER="<producer>:<round>:<kind>"`` makes producer worker
``<producer>`` fail when it starts filling round ``<round>``:

* ``exit``  -- hard crash (``os._exit(17)``, no cleanup, no error report);
* ``raise`` -- a Python exception (reported to the consumer, status FAILED);
* ``hang``  -- sleep forever (exercises the consumer's bounded waits).

``DDL_FAULT_RANK="<rank>:<window>[:<kind>]"`` makes DP rank ``<rank>``'s consumer fail when its
cursor enters global window ``<window>`` (``raise``: a Python exception; ``exit``: ``os._exit(17)``,
a silent death) -- the job-wide abort tests (``parallel/abort.py``).
"""

from __future__ import annotations

import os
import time


def _spec():
    v = os.environ.get("DDL_FAULT_PRODUCER")
    if not v:
        return None
    parts = v.split(":")
    return int(parts[0]), int(parts[1]), (parts[2] if len(parts) > 2 else "exit")


def maybe_fail_producer(index: int, rnd: int) -> None:
    spec = _spec()
    if spec is None:
        return
    p, r, kind = spec
    if p != index or r != rnd:
        return
    if kind == "exit":
        os._exit(17)
    if kind == "hang":
        while True:
            time.sleep(3600)
    raise RuntimeError(f"injected fault in producer {index} at round {rnd}")


def maybe_fail_rank(rank: int, window: int) -> None:
    v = os.environ.get("DDL_FAULT_RANK")
    if not v:
        return
    parts = v.split(":")
    if int(parts[0]) != rank or int(parts[1]) != window:
        return
    if (parts[2] if len(parts) > 2 else "raise") == "exit":
        os._exit(17)
    raise RuntimeError(f"injected fault in rank {rank} at window {window}")
