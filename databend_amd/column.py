"""DataType / Column / DataBlock for the host mirror — Databend's in-memory layout.

Mirrors `DataType`, `Column`, `DataBlock` (src/query/expression/src/types/*, values.rs:157-176,
block.rs:43-53) closely enough that a DataBlock can be handed across the C ABI without copies:
fixed-width values are little-endian numpy buffers (Decimal128 = 16-byte i128 LE), strings are a
byte buffer plus len+1 u64 offsets, validity is an arrow-style bitmap.  Device columns hold torch
tensors (torch is plumbing for device memory only).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from decimal import Decimal
from typing import List, Optional, Sequence

import numpy as np

from . import abi

_NP = {
    abi.INT8: np.int8, abi.INT16: np.int16, abi.INT32: np.int32, abi.INT64: np.int64,
    abi.UINT8: np.uint8, abi.UINT16: np.uint16, abi.UINT32: np.uint32, abi.UINT64: np.uint64,
    abi.FLOAT32: np.float32, abi.FLOAT64: np.float64, abi.DATE: np.int32, abi.TIMESTAMP: np.int64,
}
_WIDTH = {abi.INT8: 1, abi.INT16: 2, abi.INT32: 4, abi.INT64: 8, abi.UINT8: 1, abi.UINT16: 2,
          abi.UINT32: 4, abi.UINT64: 8, abi.FLOAT32: 4, abi.FLOAT64: 8, abi.DECIMAL128: 16,
          abi.DATE: 4, abi.TIMESTAMP: 8, abi.BOOLEAN: 1}
_NAMES = {abi.INT8: "Int8", abi.INT16: "Int16", abi.INT32: "Int32", abi.INT64: "Int64",
          abi.UINT8: "UInt8", abi.UINT16: "UInt16", abi.UINT32: "UInt32", abi.UINT64: "UInt64",
          abi.FLOAT32: "Float32", abi.FLOAT64: "Float64", abi.DECIMAL128: "Decimal",
          abi.DATE: "Date", abi.TIMESTAMP: "Timestamp", abi.STRING: "String",
          abi.BOOLEAN: "Boolean"}


@dataclass(frozen=True)
class DataType:
    """`DataType` (EXP/types.rs): a base type id, decimal size and the Nullable wrapper."""
    type_id: int
    precision: int = 0
    scale: int = 0
    nullable: bool = False

    def wrap_nullable(self) -> "DataType":
        return DataType(self.type_id, self.precision, self.scale, True)

    def remove_nullable(self) -> "DataType":
        return DataType(self.type_id, self.precision, self.scale, False)

    def is_nullable(self) -> bool:
        return self.nullable

    @property
    def width(self) -> int:
        return _WIDTH.get(self.type_id, 0)

    @property
    def np_dtype(self):
        return _NP.get(self.type_id)

    def to_abi(self) -> abi.dbg_datatype:
        return abi.dbg_datatype(self.type_id, self.precision, self.scale, 1 if self.nullable else 0, 0)

    @staticmethod
    def from_abi(d: abi.dbg_datatype) -> "DataType":
        return DataType(d.type, d.precision, d.scale, bool(d.nullable))

    def __repr__(self) -> str:
        n = _NAMES.get(self.type_id, str(self.type_id))
        if self.type_id == abi.DECIMAL128:
            n = f"Decimal({self.precision}, {self.scale})"
        return f"Nullable({n})" if self.nullable else n


Int8, Int16, Int32, Int64 = (DataType(t) for t in (abi.INT8, abi.INT16, abi.INT32, abi.INT64))
UInt8, UInt16, UInt32, UInt64 = (DataType(t) for t in (abi.UINT8, abi.UINT16, abi.UINT32, abi.UINT64))
Float32, Float64 = DataType(abi.FLOAT32), DataType(abi.FLOAT64)
Date, Timestamp, String, Boolean = (DataType(t) for t in (abi.DATE, abi.TIMESTAMP, abi.STRING, abi.BOOLEAN))


def Decimal128(precision: int, scale: int) -> DataType:
    return DataType(abi.DECIMAL128, precision, scale)


def pack_bits(mask: np.ndarray) -> np.ndarray:
    return np.packbits(np.asarray(mask, dtype=bool), bitorder="little")


def unpack_bits(bits: np.ndarray, n: int, offset: int = 0) -> np.ndarray:
    return np.unpackbits(np.asarray(bits, dtype=np.uint8), bitorder="little")[offset:offset + n].astype(bool)


def i128_to_bytes(values: Sequence[int]) -> np.ndarray:
    out = np.zeros(len(values) * 16, dtype=np.uint8)
    for i, v in enumerate(values):
        out[i * 16:(i + 1) * 16] = np.frombuffer(int(v).to_bytes(16, "little", signed=True), dtype=np.uint8)
    return out


def i128_from_bytes(buf: np.ndarray) -> List[int]:
    b = np.asarray(buf, dtype=np.uint8).reshape(-1, 16)
    lo = b[:, :8].copy().view(np.uint64).reshape(-1)
    hi = b[:, 8:].copy().view(np.int64).reshape(-1)
    return [int(h) * (1 << 64) + int(l) for l, h in zip(lo, hi)]


@dataclass
class Column:
    """A host Column: `data` numpy buffer (uint8 bytes for String/Decimal128, typed otherwise),
    `offsets` (String), `validity` (bool per row, None = all valid)."""
    dtype: DataType
    data: np.ndarray
    offsets: Optional[np.ndarray] = None
    validity: Optional[np.ndarray] = None
    _keep: list = field(default_factory=list, repr=False)

    def __len__(self) -> int:
        if self.dtype.type_id == abi.STRING:
            return len(self.offsets) - 1
        if self.dtype.type_id == abi.DECIMAL128:
            return len(self.data) // 16
        return len(self.data)

    # ---- constructors mirroring `XType::from_data` / `from_data_with_validity`
    @staticmethod
    def from_numbers(dtype: DataType, values, validity=None) -> "Column":
        arr = np.ascontiguousarray(np.asarray(values, dtype=dtype.np_dtype))
        v = None if validity is None else np.asarray(validity, dtype=bool)
        dt = dtype.wrap_nullable() if v is not None else dtype
        return Column(dt, arr, None, v)

    @staticmethod
    def from_strings(values: Sequence, validity=None) -> "Column":
        bs = [v.encode() if isinstance(v, str) else bytes(v) for v in values]
        offs = np.zeros(len(bs) + 1, dtype=np.uint64)
        if bs:
            offs[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
        data = np.frombuffer(b"".join(bs), dtype=np.uint8).copy() if bs else np.zeros(0, np.uint8)
        v = None if validity is None else np.asarray(validity, dtype=bool)
        return Column(String.wrap_nullable() if v is not None else String, data, offs, v)

    @staticmethod
    def from_decimals(precision: int, scale: int, values: Sequence, validity=None) -> "Column":
        """values: scaled integers (e.g. 110 for 1.10 at scale 2) or None for null."""
        if validity is None and any(x is None for x in values):
            validity = [x is not None for x in values]
        ints = [0 if x is None else int(x) for x in values]
        v = None if validity is None else np.asarray(validity, dtype=bool)
        dt = Decimal128(precision, scale)
        return Column(dt.wrap_nullable() if v is not None else dt, i128_to_bytes(ints), None, v)

    @staticmethod
    def from_bools(values: Sequence, validity=None) -> "Column":
        v = None if validity is None else np.asarray(validity, dtype=bool)
        return Column(Boolean.wrap_nullable() if v is not None else Boolean,
                      np.asarray(values, dtype=bool), None, v)

    # ---- views
    def to_abi(self) -> abi.dbg_column:
        """Borrowed dbg_column over host memory (kept alive by self._keep)."""
        c = abi.dbg_column()
        c.dt = self.dtype.to_abi()
        n = len(self)
        if self.dtype.type_id == abi.BOOLEAN:
            bits = pack_bits(self.data)
            self._keep.append(bits)
            c.data = bits.ctypes.data
        else:
            c.data = self.data.ctypes.data if self.data.size else 0
        if self.offsets is not None:
            c.offsets = self.offsets.ctypes.data
        if self.validity is not None and self.dtype.nullable:
            vb = pack_bits(self.validity)
            self._keep.append(vb)
            c.validity = vb.ctypes.data
        c.len = n
        return c

    def values(self) -> list:
        """Python values (None for null) — for comparisons in tests."""
        n = len(self)
        t = self.dtype.type_id
        if t == abi.STRING:
            out = [bytes(self.data[int(self.offsets[i]):int(self.offsets[i + 1])]) for i in range(n)]
        elif t == abi.DECIMAL128:
            out = i128_from_bytes(self.data)
        elif t == abi.BOOLEAN:
            out = [bool(x) for x in self.data]
        elif t in (abi.FLOAT32, abi.FLOAT64):
            out = [float(x) for x in self.data]
        else:
            out = [int(x) for x in self.data]
        if self.validity is not None and self.dtype.nullable:
            out = [x if ok else None for x, ok in zip(out, self.validity)]
        return out

    def decimal_values(self) -> list:
        s = self.dtype.scale
        return [None if v is None else Decimal(v).scaleb(-s) for v in self.values()]


@dataclass
class DataBlock:
    """`DataBlock` (EXP/block.rs:43-53): equal-length columns."""
    columns: List[Column]

    def num_rows(self) -> int:
        return len(self.columns[0]) if self.columns else 0

    def num_columns(self) -> int:
        return len(self.columns)


def abi_array(cols: Sequence[abi.dbg_column], ctype=abi.dbg_column):
    arr = (ctype * max(1, len(cols)))()
    for i, c in enumerate(cols):
        arr[i] = c
    return arr
