"""One device-side total order for every collective a rank issues.

The reference's cross-GPU exchange runs on its own MPI communicator
(``comm_nth_pusher``, reference ddl/ddl_env.py:74-81, ddl/shuffle.py:92-108)
and training traffic on the user's torch.distributed group; MPI progresses
them on the host, so two communicators cannot deadlock each other there.

On MI355X both are RCCL kernels. A collective kernel spins until its peers
arrive, and with ``GPU_MAX_HW_QUEUES=4`` the runtime multiplexes more streams
than that onto 4 in-order hardware queues. Two communicators on two streams
can therefore deadlock across ranks: rank 0's queue holds the loader's
all-to-all in front of DDP's all-reduce while rank 1's holds them the other
way round, and each kernel waits for a peer that sits behind the other one.

The invariant used here removes that hazard by construction:

1. **One communicator.** The loader's exchange (``parallel/shuffle.py``) and
   the resident loader's all-to-all (``resident.py``) are issued on the DP
   process group (:func:`loader_group`), the same group the trainer hands to
   DDP. ProcessGroupNCCL runs every collective of a group (and batched P2P)
   on one ncclComm and one internal stream per device, so their device-side
   order is their issue order.
2. **One issuing thread in program order.** Every loader collective is issued
   by the consumer thread at a fixed point of the batch schedule (window
   ``w+1``'s exchange when window ``w`` is handed back at its last
   ``END_OF_BATCH``, ``dataloader._begin_window`` / ``staging.post``), never by
   the native stager thread, whose progress depends on producer timing. DDP's
   bucket all-reduces are launched while the same thread is blocked in
   ``backward()``, in bucket order. So the issue order is a function of the
   step/window schedule only, and it is identical on every rank.

:data:`LEDGER` records the issue sequence (kind, key) when enabled, and
:func:`check_same_order` compares a digest of it across ranks; the tests and
``bench.py`` use this to check the invariant on real runs.
"""

from __future__ import annotations

import hashlib
import os
import threading


class CollectiveLedger:
    """Append-only log of (kind, key) for every collective issued by this process."""

    def __init__(self) -> None:
        self.enabled = os.environ.get("DDL_TRACE_COLLECTIVES", "0") == "1"
        self.entries: list[tuple[str, object]] = []
        self.threads: set[int] = set()

    def enable(self, on: bool = True) -> None:
        self.enabled = on

    def clear(self) -> None:
        self.entries.clear()
        self.threads.clear()

    def record(self, kind: str, key: object = None) -> None:
        if self.enabled:
            self.entries.append((kind, key))
            self.threads.add(threading.get_ident())

    def digest(self) -> str:
        h = hashlib.sha1()
        for kind, key in self.entries:
            h.update(f"{kind}:{key};".encode())
        return h.hexdigest()

    def counts(self) -> dict[str, int]:
        out: dict[str, int] = {}
        for kind, _ in self.entries:
            out[kind] = out.get(kind, 0) + 1
        return out


LEDGER = CollectiveLedger()


def loader_group(env):
    """The process group the loader issues its collectives on: the DP group itself (see module doc)."""
    return env.process_group


def ddp_ledger_hook(process_group):
    """DDP comm hook: the default bucket all-reduce, recorded in :data:`LEDGER` at issue."""
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks

    def hook(state, bucket):
        LEDGER.record("ddp.allreduce", bucket.index())
        return default_hooks.allreduce_hook(process_group, bucket)

    return hook


def check_same_order(control_group) -> dict:
    """All-gather the ledger digest over the (gloo) control group.

    Returns ``{"same_order", "n_collectives", "by_kind", "issuing_threads"}``;
    ``same_order`` is True when every rank issued the same sequence.
    """
    import torch.distributed as dist

    mine = (LEDGER.digest(), len(LEDGER.entries))
    out = {"same_order": True, "n_collectives": mine[1], "by_kind": LEDGER.counts(),
           "issuing_threads": len(LEDGER.threads)}
    if control_group is None or not dist.is_initialized():
        return out
    allv: list = [None] * dist.get_world_size(control_group)
    dist.all_gather_object(allv, mine, group=control_group)
    out["same_order"] = len({d for d, _ in allv}) == 1
    return out
