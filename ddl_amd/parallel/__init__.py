"""Parallelism: rank topology, launcher, cross-GPU global shuffle (RCCL/xGMI)."""

from .env import init_distributed, init_mpi, init_mpi_error_handling, read_env
from .launcher import distributed_dataloader, spawn_producers, start
from .shuffle import (
    AllToAllGlobalShuffler,
    GlobalShuffler,
    SendRecvReplaceGlobalShuffler,
    derangement_partners,
    make_exchange,
)

__all__ = [
    "init_distributed",
    "init_mpi",
    "init_mpi_error_handling",
    "read_env",
    "distributed_dataloader",
    "spawn_producers",
    "start",
    "AllToAllGlobalShuffler",
    "GlobalShuffler",
    "SendRecvReplaceGlobalShuffler",
    "derangement_partners",
    "make_exchange",
]
