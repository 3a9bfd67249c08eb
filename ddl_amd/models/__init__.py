"""Dataset / producer families and the synthetic train steps used by the benches."""

from .datasets import (
    DummyDataset,
    FileRowsSource,
    MapDatasetSource,
    NpyMemmapSource,
    PointWiseData,
    SharedArraySource,
    SyntheticTokens,
    synthetic_images,
    numa_local_source,
    unpack_fields,
)
from .producers import ImageWindowProducer, IndexedProducer, PointwiseProducer

__all__ = [
    "DummyDataset",
    "FileRowsSource",
    "MapDatasetSource",
    "NpyMemmapSource",
    "PointWiseData",
    "SharedArraySource",
    "SyntheticTokens",
    "synthetic_images",
    "numa_local_source",
    "unpack_fields",
    "ImageWindowProducer",
    "IndexedProducer",
    "PointwiseProducer",
]
