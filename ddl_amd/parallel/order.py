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
2. **One issue order, a function of the schedule only.** Every loader
   collective is issued by the consumer thread at a fixed point of the batch
   schedule (window ``w+1``'s exchange when the cursor enters window ``w``,
   ``dataloader._ensure_posted`` / ``staging.post``), never by the native
   stager thread, whose progress depends on producer timing. DDP's bucket
   all-reduces are issued from autograd's device thread (the ledger reports
   ``issuing_threads: 2``), but only while the consumer thread is blocked in
   ``backward()``, in bucket order, so the two threads never issue
   concurrently: the issue order is a function of the step/window schedule
   and identical on every rank.
3. **Enforced, not assumed.** Every loader collective and point-to-point
   batch goes through :func:`issue` / :func:`check_group`, which raise
   :class:`~ddl_amd.exceptions.CommunicatorMismatchError` if the group is not
   ``env.process_group`` itself; the ledger records the group of every entry
   (DDP's hook included) and :func:`check_same_order` reports how many
   distinct groups were used (1 when the invariant holds).

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
        self.groups: set[str] = set()

    def enable(self, on: bool = True) -> None:
        self.enabled = on

    def clear(self) -> None:
        self.entries.clear()
        self.threads.clear()
        self.groups.clear()

    def record(self, kind: str, key: object = None, group=None) -> None:
        if self.enabled:
            self.entries.append((kind, key))
            self.threads.add(threading.get_ident())
            if group is not None:
                self.groups.add(group_id(group))

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


def group_id(group) -> str:
    """A stable name of a process group (its c10d name; the object id if it has none)."""
    name = getattr(group, "group_name", None)
    return str(name) if name else f"obj:{id(group):x}"


def loader_group(env):
    """The process group the loader issues its collectives on: the DP group itself (see module doc)."""
    return env.process_group


def check_group(env, group, what: str) -> None:
    """Raise unless ``group`` is the DP group ``env.process_group`` itself (the same object: the same
    ncclComm and stream as the trainer's DDP all-reduce)."""
    if group is None or group is not env.process_group:
        from ..exceptions import CommunicatorMismatchError

        raise CommunicatorMismatchError(
            (what, group_id(group) if group is not None else None,
             group_id(env.process_group) if env.process_group is not None else None),
            f"{what}: loader collectives must be issued on the DP process group (env.process_group), so that "
            f"they share one communicator and device order with DDP (parallel/order.py); got another group")


def issue(env, group, kind: str, key: object = None) -> None:
    """Gate of every loader collective: check the group, then record (kind, key, group) in the ledger."""
    check_group(env, group, kind)
    LEDGER.record(kind, key, group)


def ddp_ledger_hook(process_group):
    """DDP comm hook: the default bucket all-reduce, recorded in :data:`LEDGER` at issue (with its group)."""
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks

    def hook(state, bucket):
        LEDGER.record("ddp.allreduce", bucket.index(), process_group)
        return default_hooks.allreduce_hook(process_group, bucket)

    return hook


def check_same_order(control_group) -> dict:
    """All-gather the ledger digest over the (gloo) control group.

    Returns ``{"same_order", "n_collectives", "by_kind", "issuing_threads", "groups"}``;
    ``same_order`` is True when every rank issued the same sequence, ``groups`` is the number of
    distinct process groups the recorded collectives were issued on (1: one communicator).
    """
    import torch.distributed as dist

    mine = (LEDGER.digest(), len(LEDGER.entries))
    out = {"same_order": True, "n_collectives": mine[1], "by_kind": LEDGER.counts(),
           "issuing_threads": len(LEDGER.threads), "groups": len(LEDGER.groups)}
    if control_group is None or not dist.is_initialized():
        return out
    allv: list = [None] * dist.get_world_size(control_group)
    dist.all_gather_object(allv, mine, group=control_group)
    out["same_order"] = len({d for d, _ in allv}) == 1
    return out
