"""Device-resident columns (HBM) as torch tensors — plumbing for the C ABI's on_device path.

`DeviceColumn.to_abi()` yields a `dbg_column` whose pointers are HBM addresses; the kernels read
them in place.  torch provides allocation and streams only.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi
from .column import Column, DataType, pack_bits


def _torch():
    import torch
    return torch


@dataclass
class DeviceColumn:
    dtype: DataType
    data: "object"                     # torch uint8/typed tensor on cuda
    offsets: Optional["object"] = None  # torch int64 tensor (u64 offsets) for strings
    validity: Optional["object"] = None  # torch uint8 tensor, arrow bitmap
    length: int = 0
    _keep: list = field(default_factory=list, repr=False)

    def __len__(self):
        return self.length

    def to_abi(self) -> abi.dbg_column:
        c = abi.dbg_column()
        c.dt = self.dtype.to_abi()
        c.data = self.data.data_ptr() if self.data is not None and self.data.numel() else 0
        if self.offsets is not None:
            c.offsets = self.offsets.data_ptr()
        if self.validity is not None and self.dtype.nullable:
            c.validity = self.validity.data_ptr()
        c.len = self.length
        return c

    @staticmethod
    def from_host(col: Column, device="cuda") -> "DeviceColumn":
        torch = _torch()
        n = len(col)
        if col.dtype.type_id == abi.BOOLEAN:
            data = torch.from_numpy(pack_bits(col.data)).to(device)
        else:
            data = torch.from_numpy(np.ascontiguousarray(col.data).view(np.uint8).copy()).to(device)
        offs = None
        if col.offsets is not None:
            offs = torch.from_numpy(col.offsets.astype(np.uint64).view(np.int64).copy()).to(device)
        val = None
        if col.validity is not None and col.dtype.nullable:
            val = torch.from_numpy(pack_bits(col.validity)).to(device)
        return DeviceColumn(col.dtype, data, offs, val, n)

    def to_host(self) -> Column:
        n = self.length
        raw = self.data.cpu().numpy()
        t = self.dtype.type_id
        offs = self.offsets.cpu().numpy().view(np.uint64) if self.offsets is not None else None
        if t == abi.BOOLEAN:
            data = np.unpackbits(raw, bitorder="little")[:n].astype(bool)
        elif t in (abi.STRING, abi.DECIMAL128):
            data = raw
        else:
            data = raw.view(self.dtype.np_dtype)[:n]
        val = None
        if self.validity is not None and self.dtype.nullable:
            val = np.unpackbits(self.validity.cpu().numpy(), bitorder="little")[:n].astype(bool)
        return Column(self.dtype, data, offs, val)


def empty(dtype: DataType, n: int, device="cuda", string_bytes: int = 0) -> DeviceColumn:
    torch = _torch()
    if dtype.type_id == abi.STRING:
        data = torch.empty(max(1, string_bytes), dtype=torch.uint8, device=device)
        offs = torch.empty(n + 1, dtype=torch.int64, device=device)
    else:
        w = dtype.width if dtype.type_id != abi.BOOLEAN else 1
        data = torch.empty(max(1, n * w), dtype=torch.uint8, device=device)
        offs = None
    val = torch.empty(max(1, (n + 7) // 8), dtype=torch.uint8, device=device) if dtype.nullable else None
    return DeviceColumn(dtype, data, offs, val, n)
