"""Hook protocol of the producer pipeline (reference ddl/protocols.py:4-18).

The reference protocol names ``exec_function`` while the data pusher dispatches
``execute_function`` (reference ddl/protocols.py:11 vs ddl/datapusher.py:154);
here the protocol and the dispatcher agree on ``execute_function``.
"""

from __future__ import annotations

from typing import Any, Protocol, runtime_checkable

#: Hook names in the order the producer engine dispatches them.
HOOKS = (
    "on_init",
    "post_init",
    "on_push_begin",
    "global_shuffle",
    "execute_function",
    "on_shuffle_end",
    "on_push_end",
)


@runtime_checkable
class CallbackProtocol(Protocol):
    def on_push_begin(self, **kwargs: Any) -> Any: ...

    def global_shuffle(self, **kwargs: Any) -> Any: ...

    def execute_function(self, **kwargs: Any) -> Any: ...

    def on_push_end(self, **kwargs: Any) -> Any: ...

    def on_shuffle_end(self, **kwargs: Any) -> Any: ...
