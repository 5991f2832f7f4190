"""databend_amd — an MI355X-native filter + hash GROUP BY path for Databend.

The product is libdbgpu_agg.so (HIP kernels for gfx950 behind the C ABI in include/dbgpu_agg.h).
This package is the host-side mirror of the reference's operator interface for that path
(TransformPartialAggregate / TransformFinalAggregate / AggregateFunction / TransformFilter) over
ctypes, plus the multi-GPU exchange over torch.distributed (RCCL).
"""
from .column import Column, DataBlock, DataType  # noqa: F401

__all__ = ["Column", "DataBlock", "DataType"]
