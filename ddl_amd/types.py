"""Records exchanged between consumer and producers, and the process environment.

Mirrors reference ddl/types.py:7-37 (+ ddl/connection.py:12-14 ``WorkerInfo``)
with the fields the reference lacks: dtype, seed, epoch/sample cursor, slot
count and the producer's pid (for liveness checks).
"""

from __future__ import annotations

import dataclasses
from enum import Enum, auto
from typing import Any


class Marker(Enum):
    """Consumer state-machine events (reference ddl/types.py:35-37)."""

    END_OF_BATCH = auto()
    END_OF_EPOCH = auto()


class WorkerInfo(Enum):
    """Producer loop control (reference ddl/connection.py:12-14)."""

    CONTINUE = auto()
    STOP = auto()


@dataclasses.dataclass
class MetaData_Consumer_To_Producer:  # noqa: N801  (reference name)
    producer_function: Any
    global_shuffle_fraction_exchange: float
    global_shuffle_exchange_method: str
    batch_size: int
    # --- additions ---
    producer_index: int = 0
    n_producers: int = 1
    rank: int = 0
    world_size: int = 1
    n_slots: int = 1
    seed: int = 0
    start_round: int = 0
    host_threads: int = 4


@dataclasses.dataclass
class MetaData_Producer_To_Consumer:  # noqa: N801  (reference name)
    nData: int  # noqa: N815
    nValues: int  # noqa: N815
    shape: tuple[int, ...]
    splits: tuple[int, ...]
    batches_per_window: int
    # --- additions ---
    dtype: str = "float32"
    pid: int = 0
    extra: dict = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class DDLEnv:
    """Process environment of one consumer (= one DP rank = one GPU).

    Replaces the reference's ``MPI_Env`` of four communicators
    (reference ddl/types.py:24-32): ranks come from torchrun / SLURM env
    variables, the DP group is a torch.distributed group (RCCL on GPU, gloo on
    CPU) and the per-GPU producers are child processes, not ranks.
    """

    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    node_rank: int = 0
    n_producers: int = 0
    hostname: str = ""
    device: str = ""  # set by init_distributed ("cuda:<i>" or "cpu"); "" = not chosen yet
    backend: str | None = None
    process_group: Any = None  # DP group (RCCL on GPU); None when world_size == 1
    control_group: Any = None  # gloo group for host-side control traffic

    # reference-compatible aliases (ddl/types.py:24-32)
    @property
    def n_instances(self) -> int:
        return self.world_size

    @property
    def color(self) -> int:
        return self.rank

    @property
    def color_nth_pusher(self) -> int:
        return 0

    @property
    def comm_global(self) -> Any:
        """The reference's WORLD communicator: the DP process group (None for a single rank)."""
        return self.process_group

    @property
    def comm_nth_pusher(self) -> Any:
        """The reference's k-th-pusher communicator, over which its GPUs exchange rows
        (ddl/ddl_env.py:74-81). Here the consumers exchange on the DP group."""
        return self.process_group

    @property
    def comm_per_gpu(self) -> None:
        """No per-GPU communicator: a rank's producers are its child processes."""
        return None

    comm_per_gpu_shm = comm_per_gpu


MPI_Env = DDLEnv  # reference name (ddl/types.py:24-32)
