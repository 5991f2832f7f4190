"""ORDER BY <columns> [ASC|DESC] [NULLS FIRST|LAST] LIMIT k on device.

Host mirror of `DataBlock::sort(block, descriptions, limit)` (EXP/kernels/sort.rs:79-107) for one
sort column — the shape that ends every ClickBench GROUP BY query (`ORDER BY c DESC LIMIT 10`),
run over the aggregate's result columns while they are still in HBM.  The indices come from
`dbg_sort_limit_indices` (databend_amd/csrc/sort.hip: radix select + LDS bitonic sort); the
columns are gathered with `dbg_take_fixed` (DataBlock::take, EXP/kernels/take.rs:56-91).

Semantics follow arrow's sort_to_indices (src/common/arrow/src/arrow/compute/sort/common.rs:95-174):
NULLs first or last in ascending row order, integer order / IEEE totalOrder for floats, DESC
reverses the value order only.  Equal values come out in ascending row order (the reference's
select_nth_unstable_by leaves them unspecified).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence

from . import abi
from .device import DeviceColumn, empty
from .ffi import check, lib

SORT_LIMIT_MAX = 2048  # SORT_CAP in csrc/sort.hpp


@dataclass
class SortColumnDescription:
    """EXP/kernels/sort.rs:50-56."""
    offset: int
    asc: bool = True
    nulls_first: bool = False
    is_nullable: bool = False


def sort_limit_indices(col: DeviceColumn, asc: bool, nulls_first: bool, limit: Optional[int]):
    """Row indices (torch int32 on the column's device) of the first min(limit, rows) rows."""
    import torch

    n = len(col)
    k = n if limit is None else min(int(limit), n)
    out = torch.empty(max(1, k), dtype=torch.int32, device=col.data.device)
    got = C.c_uint64()
    check(lib().dbg_sort_limit_indices(C.byref(col.to_abi()), n, 1 if asc else 0, 1 if nulls_first else 0, k,
                                       out.data_ptr(), C.byref(got), None))
    return out[:got.value]


def take(col: DeviceColumn, idx) -> DeviceColumn:
    """DataBlock::take of one column by device u32 indices (EXP/kernels/take.rs:56-91):
    dbg_take_fixed for fixed-width columns, dbg_take_string for strings."""
    n = int(idx.numel())
    if col.dtype.type_id == abi.STRING:
        cap = max(1, int(col.data.numel()))
        out = empty(col.dtype, n, device=col.data.device, string_bytes=cap)
        total = C.c_uint64()
        check(lib().dbg_take_string(C.byref(col.to_abi()), idx.data_ptr() if n else None, n, out.offsets.data_ptr(),
                                    out.data.data_ptr(), cap,
                                    out.validity.data_ptr() if out.validity is not None else None, C.byref(total), None))
        out.data = out.data[: max(1, total.value)]
        return out
    out = empty(col.dtype, n, device=col.data.device)
    check(lib().dbg_take_fixed(C.byref(col.to_abi()), idx.data_ptr(), n, out.data.data_ptr(),
                               out.validity.data_ptr() if out.validity is not None else None, None))
    return out


def sort_multi_limit_indices(columns: Sequence[DeviceColumn], descriptions: Sequence[SortColumnDescription],
                             limit: Optional[int]):
    """Row indices (torch int32) of the first min(limit, rows) rows in the order of several sort
    columns — numbers, Decimal128 or String, each with its own direction (dbg_sort_limit_multi)."""
    import torch

    cols = [columns[d.offset] for d in descriptions]
    n = len(cols[0])
    k = n if limit is None else min(int(limit), n)
    arr = (abi.dbg_column * len(cols))(*[c.to_abi() for c in cols])
    asc = (C.c_int * len(cols))(*[1 if d.asc else 0 for d in descriptions])
    nf = (C.c_int * len(cols))(*[1 if d.nulls_first else 0 for d in descriptions])
    out = torch.empty(max(1, k), dtype=torch.int32, device=cols[0].data.device)
    got = C.c_uint64()
    check(lib().dbg_sort_limit_multi(arr, len(cols), asc, nf, n, k, out.data_ptr(), C.byref(got), None))
    return out[:got.value]


def sort(columns: Sequence[DeviceColumn], descriptions: Sequence[SortColumnDescription],
         limit: Optional[int]) -> List[DeviceColumn]:
    """DataBlock::sort (EXP/kernels/sort.rs:79-107): one fixed-width number column takes the
    radix-select path of dbg_sort_limit_indices; several columns, or a String / Decimal128 one,
    the composite-key path of dbg_sort_limit_multi."""
    if not descriptions:
        raise ValueError("sort: no sort description")
    d = descriptions[0]
    one_number = len(descriptions) == 1 and columns[d.offset].dtype.type_id not in (abi.STRING, abi.DECIMAL128)
    if one_number:
        idx = sort_limit_indices(columns[d.offset], d.asc, d.nulls_first, limit)
    else:
        idx = sort_multi_limit_indices(columns, descriptions, limit)
    return [take(c, idx) for c in columns]
