"""dtype codes shared with csrc/kernels/common.h (enum DType)."""

from __future__ import annotations

import numpy as np
import torch

U8, I32, I64, F16, BF16, F32 = 0, 1, 2, 3, 4, 5

_TORCH_TO_CODE = {
    torch.uint8: U8,
    torch.int32: I32,
    torch.int64: I64,
    torch.float16: F16,
    torch.bfloat16: BF16,
    torch.float32: F32,
}

_NAME_TO_TORCH = {
    "uint8": torch.uint8,
    "u8": torch.uint8,
    "int16": torch.int16,
    "int32": torch.int32,
    "int64": torch.int64,
    "float16": torch.float16,
    "fp16": torch.float16,
    "half": torch.float16,
    "bfloat16": torch.bfloat16,
    "bf16": torch.bfloat16,
    "float32": torch.float32,
    "fp32": torch.float32,
    "float": torch.float32,
}


def code(dtype: torch.dtype) -> int:
    try:
        return _TORCH_TO_CODE[dtype]
    except KeyError:
        raise TypeError(f"dtype {dtype} is not supported by the ddl_amd kernels") from None


def to_torch_dtype(dt) -> torch.dtype:
    """Accept a torch dtype, numpy dtype, or name ('bf16', 'float32', ...)."""
    if isinstance(dt, torch.dtype):
        return dt
    if isinstance(dt, str):
        try:
            return _NAME_TO_TORCH[dt.lower()]
        except KeyError:
            raise TypeError(f"unknown dtype name {dt!r}") from None
    npd = np.dtype(dt)
    m = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int16): torch.int16, np.dtype(np.int32): torch.int32,
         np.dtype(np.int64): torch.int64, np.dtype(np.float16): torch.float16, np.dtype(np.float32): torch.float32}
    if npd in m:
        return m[npd]
    raise TypeError(f"unsupported dtype {dt!r}")


def numpy_view_dtype(dt: torch.dtype):
    """numpy dtype for a host view of ``dt`` (bf16 has none: returns None)."""
    m = {torch.uint8: np.uint8, torch.int16: np.int16, torch.int32: np.int32, torch.int64: np.int64,
         torch.float16: np.float16, torch.float32: np.float32}
    return m.get(dt)


def itemsize(dt: torch.dtype) -> int:
    return torch.empty((), dtype=dt).element_size()
