"""User extension point: the producer function (reference ddl/datasetwrapper.py:4-19).

Same hook names and semantics as the reference. The object is constructed on
the consumer and pickled to every producer worker process (reference
ddl/connection.py:72-73), so it must stay picklable; its hooks run in the
producer process, which never touches the GPU.

Hooks (all optional except ``execute_function``; all called with keyword
arguments):

``on_init(rank_global=..., producer_index=..., n_producers=..., ...)``
    load/generate the shard; must return a ``DataProducerOnInitReturn``.
``post_init(my_ary=..., my_tensor=..., ...)``
    fill the window (``my_ary``: numpy view when the dtype has one, else the
    torch view; ``my_tensor``: torch view of the same memory).
``execute_function(my_ary=..., round=..., ...)``
    refill / re-shuffle the window in place before each publish.
``on_push_begin``, ``on_shuffle_end``, ``on_push_end``, ``global_shuffle``.
"""

from __future__ import annotations

import os
from typing import Any


class ProducerFunctionSkeleton:
    # Pinned slots per producer the loader uses when its ``n_slots`` is not given. One slot suffices when a
    # round is cheap (the slot is back with its producer as soon as its H2D copy retires); a producer that
    # rewrites its whole window every round sets 2, so one slot is refilled while the other is copied
    # (archive/profiles/r3_full_refill: 141k -> 175-178k samples/s).
    preferred_slots: int = 1

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        self.my_ary = None
        self.my_tensor = None
        self.rank_global: int | None = None
        self.producer_index: int | None = None
        self.n_producers: int | None = None

    def on_init(self, *args: Any, **kwargs: Any) -> Any:
        # reference falls back to COMM_WORLD.Get_rank(); we fall back to RANK.
        self.rank_global = kwargs.get("rank_global", int(os.environ.get("RANK", "0") or 0))
        self.producer_index = kwargs.get("producer_index", self.producer_index)
        self.n_producers = kwargs.get("n_producers", self.n_producers)
        return None

    def post_init(self, *args: Any, **kwargs: Any) -> Any:
        self.my_ary = kwargs["my_ary"]
        self.my_tensor = kwargs.get("my_tensor")
        return None

    def execute_function(self, *args: Any, **kwargs: Any) -> Any:
        raise NotImplementedError
