"""Dataset / producer families and the synthetic train steps used by the benches."""

from .datasets import (
    DummyDataset,
    FileRowsSource,
    NpyMemmapSource,
    PointWiseData,
    SharedArraySource,
    SyntheticTokens,
    synthetic_images,
)
from .producers import ImageWindowProducer, IndexedProducer, PointwiseProducer

__all__ = [
    "DummyDataset",
    "FileRowsSource",
    "NpyMemmapSource",
    "PointWiseData",
    "SharedArraySource",
    "SyntheticTokens",
    "synthetic_images",
    "ImageWindowProducer",
    "IndexedProducer",
    "PointwiseProducer",
]
