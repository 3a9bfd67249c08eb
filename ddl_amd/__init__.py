"""ddl_amd -- an MI355X-native distributed data loader for PyTorch-ROCm.

Capabilities and drop-in API of ``maximilian-tech/ddl`` (same five public
names, reference ddl/__init__.py:7-21), re-designed for MI355X: C++ shm slot
runtime instead of MPI windows, pinned H2D staging on a prefetch HIP stream,
hand-written gfx950 kernels for permute/cast/collate/pad-pack, RCCL over xGMI
for the cross-GPU global shuffle, world-size-invariant deterministic order.
"""

__all__ = [
    "ProducerFunctionSkeleton",
    "DataProducerOnInitReturn",
    "distributed_dataloader",
    "DistributedDataLoader",
    "Marker",
    # additions
    "DDLEnv",
    "start",
    "FeistelPermutation",
    "EpochOrder",
    "IndexedProducer",
    "DataLoader",
    "OutputSpec",
    "StagingSpec",
    "OrderSpec",
    "ops",
]

from . import ops
from .datapusher import DataProducerOnInitReturn
from .dataloader import DistributedDataLoader
from .datasetwrapper import ProducerFunctionSkeleton
from .parallel.launcher import distributed_dataloader, start
from .permutation import EpochOrder, FeistelPermutation
from .specs import OrderSpec, OutputSpec, StagingSpec
from .types import DDLEnv, Marker


def __getattr__(name):
    if name == "IndexedProducer":
        from .models.producers import IndexedProducer

        return IndexedProducer
    if name == "DataLoader":
        from .frontend import DataLoader

        return DataLoader
    raise AttributeError(name)
