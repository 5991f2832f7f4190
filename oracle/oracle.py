"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/liboracle.so, the C++ restatement of Databend's filter + hash GROUP BY
(oracle/dbagg_oracle.cpp).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module; the product package databend_amd never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

from databend_amd import abi
from databend_amd.column import Column, DataType, abi_array, unpack_bits

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_last_error.restype = C.c_char_p
        L.orc_result_rows.restype = C.c_uint64
        L.orc_result_rows.argtypes = [C.c_void_p]
        L.orc_result_free.argtypes = [C.c_void_p]
        L.orc_result_column.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(abi.dbg_datatype),
                                        C.POINTER(C.c_void_p), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.orc_aggregate.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                    C.c_uint64, C.c_int, C.POINTER(C.c_void_p)]
        L.orc_aggregate_serialized.argtypes = L.orc_aggregate.argtypes
        L.orc_merge_serialized.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_uint64, C.c_int,
                                           C.POINTER(C.c_void_p)]
        L.orc_group_hash.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_void_p]
        L.orc_legacy_group_hash.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_void_p]
        L.orc_crc32c_bytes.argtypes = [C.c_uint32, C.c_void_p, C.c_uint64]
        L.orc_crc32c_bytes.restype = C.c_uint32
        L.orc_filter_select.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.POINTER(C.c_uint64)]
        L.orc_datagen.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_datagen_c5_bytes.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_int]
        L.orc_c5_cdf.argtypes = [C.c_void_p]
        L.orc_result_type.argtypes = [C.c_void_p, C.c_void_p]
        _LIB = L
    return _LIB


class OracleError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"oracle error {code}: {msg}")
        self.code = code


def _check(rc: int):
    if rc != 0:
        raise OracleError(rc, lib().orc_last_error().decode())


def group_hash(cols: Sequence[Column]) -> np.ndarray:
    """group_hash_columns (EAGG/group_hash.rs:41-48)."""
    n = len(cols[0])
    out = np.zeros(n, dtype=np.uint64)
    arr = abi_array([c.to_abi() for c in cols])
    _check(lib().orc_group_hash(arr, len(cols), n, out.ctypes.data))
    return out


def legacy_group_hash(cols: Sequence[Column]) -> np.ndarray:
    """FastHash of the legacy HashMethod key (FixedKeys / SingleBinary), HT/traits.rs:172-330."""
    n = len(cols[0])
    out = np.zeros(max(1, n), dtype=np.uint64)
    arr = abi_array([c.to_abi() for c in cols])
    _check(lib().orc_legacy_group_hash(arr, len(cols), n, out.ctypes.data))
    return out[:n]


def crc32c(data: bytes, crc: int = 0xFFFFFFFF) -> int:
    """Raw CRC32C update (no final inversion) of `data` from `crc`."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if data else np.zeros(1, np.uint8)
    return int(lib().orc_crc32c_bytes(crc, buf.ctypes.data, len(data)))


def result_type(spec: abi.dbg_agg_spec) -> DataType:
    out = abi.dbg_datatype()
    _check(lib().orc_result_type(C.byref(spec), C.byref(out)))
    return DataType.from_abi(out)


def filter_select(program, rows: int) -> np.ndarray:
    sel = np.zeros(max(1, rows), dtype=np.uint32)
    n = C.c_uint64()
    _check(lib().orc_filter_select(program.ptr(), rows, sel.ctypes.data, C.byref(n)))
    return sel[:n.value].copy()


def _to_column(r, which: int, idx: int, rows: int) -> Column:
    dt = abi.dbg_datatype()
    data, nbytes, offs, valid = C.c_void_p(), C.c_uint64(), C.c_void_p(), C.c_void_p()
    _check(lib().orc_result_column(r, which, idx, C.byref(dt), C.byref(data), C.byref(nbytes),
                                   C.byref(offs), C.byref(valid)))
    d = DataType.from_abi(dt)
    raw = np.ctypeslib.as_array((C.c_uint8 * max(1, nbytes.value)).from_address(data.value))[:nbytes.value].copy() \
        if nbytes.value else np.zeros(0, np.uint8)
    v = np.ctypeslib.as_array((C.c_uint8 * max(1, rows)).from_address(valid.value))[:rows].astype(bool).copy() \
        if rows else np.zeros(0, bool)
    offsets = None
    if d.type_id == abi.STRING:
        offsets = np.ctypeslib.as_array((C.c_uint64 * (rows + 1)).from_address(offs.value)).copy()
        data_arr = raw
    elif d.type_id == abi.DECIMAL128:
        data_arr = raw
    elif d.type_id == abi.BOOLEAN:
        data_arr = raw.astype(bool)
    else:
        data_arr = raw.view(d.np_dtype).copy()
    return Column(d, data_arr, offsets, v if d.nullable else None)


def _collect(out, n_keys: int, n_aggs: int):
    try:
        rows = lib().orc_result_rows(out)
        kc = [_to_column(out, 0, i, rows) for i in range(n_keys)]
        ac = [_to_column(out, 1, i, rows) for i in range(n_aggs)]
    finally:
        lib().orc_result_free(out)
    return kc, ac


def aggregate(keys: Sequence[Column], aggs: Sequence[Tuple[abi.dbg_agg_spec, Optional[Column]]],
              filter_program=None, threads: int = 1, serialize: bool = False) -> Tuple[List[Column], List[Column]]:
    """Run the restated pipeline (partial x threads -> bucket -> final).  Returns (keys, aggs);
    serialize=True returns each aggregate's final state as a Binary column of borsh bytes
    (AggregateMeta::Serialized's state columns) instead of its result."""
    n = len(keys[0])
    karr = abi_array([k.to_abi() for k in keys])
    arg_structs = []
    for spec, col in aggs:
        if col is None:
            c = abi.dbg_column()
            c.dt = abi.dbg_datatype(-1, 0, 0, 0, 0)
            arg_structs.append(c)
        else:
            arg_structs.append(col.to_abi())
    aarr = abi_array(arg_structs)
    sarr = abi_array([s for s, _ in aggs], abi.dbg_agg_spec)
    out = C.c_void_p()
    fn = lib().orc_aggregate_serialized if serialize else lib().orc_aggregate
    _check(fn(karr, len(keys), aarr, sarr, len(aggs), filter_program.ptr() if filter_program is not None else None,
              n, threads, C.byref(out)))
    return _collect(out, len(keys), len(aggs))


def merge_serialized(keys: Sequence[Column], states: Sequence[Column], specs: Sequence[abi.dbg_agg_spec],
                     serialize: bool = False) -> Tuple[List[Column], List[Column]]:
    """TransformFinalAggregate over one AggregateMeta::Serialized block (group columns + Binary
    state columns): re-insert with batch_merge, then merge_result (or serialize again)."""
    n = len(keys[0])
    karr = abi_array([k.to_abi() for k in keys])
    st = abi_array([c.to_abi() for c in states]) if states else None
    sarr = abi_array(list(specs), abi.dbg_agg_spec) if specs else None
    out = C.c_void_p()
    _check(lib().orc_merge_serialized(karr, len(keys), st, sarr, len(specs), n, 1 if serialize else 0, C.byref(out)))
    return _collect(out, len(keys), len(specs))


# ---- CPU workload generator (include/dbgpu_datagen.h) ----
_C5_CDF = None


def c5_cdf() -> np.ndarray:
    global _C5_CDF
    if _C5_CDF is None:
        cdf = np.zeros(1 << 23, dtype=np.uint64)
        lib().orc_c5_cdf(cdf.ctypes.data)
        _C5_CDF = cdf
    return _C5_CDF


def datagen(cfg: int, rows: int, start: int = 0, seed: Optional[int] = None, threads: int = 8) -> dict:
    """Columns of config cfg for rows [start, start+rows) as host Columns (names as in DESIGN.md)."""
    from databend_amd import column as col
    seed = (0xDA7ABE7D + cfg) if seed is None else seed
    L = lib()
    if cfg == 1:
        bufs = [np.zeros(rows, np.int32), np.zeros(rows, np.uint8), np.zeros(rows, np.uint8)] + \
               [np.zeros(rows, np.int64) for _ in range(6)]
        ptrs = (C.c_void_p * 9)(*[b.ctypes.data for b in bufs])
        _check(L.orc_datagen(1, seed, start, rows, ptrs, None, threads))
        ar = np.arange(rows + 1, dtype=np.uint64)

        def dec(a, p, s):
            b = np.zeros((rows, 16), np.uint8)
            b[:, :8] = a.view(np.uint8).reshape(rows, 8)
            b[:, 8:] = np.where(a < 0, 0xFF, 0).astype(np.uint8)[:, None]
            return Column(col.Decimal128(p, s), b.reshape(-1))

        return {
            "l_shipdate": Column(col.Date, bufs[0]),
            "l_returnflag": Column(col.String, bufs[1], ar.copy()),
            "l_linestatus": Column(col.String, bufs[2], ar.copy()),
            "l_quantity": dec(bufs[3], 15, 2),
            "l_extendedprice": dec(bufs[4], 15, 2),
            "l_discount": dec(bufs[5], 15, 2),
            "l_tax": dec(bufs[6], 15, 2),
            "disc_price": dec(bufs[7], 31, 4),
            "charge": dec(bufs[8], 38, 6),
        }
    if cfg == 2:
        b = np.zeros(rows, np.int16)
        _check(L.orc_datagen(2, seed, start, rows, (C.c_void_p * 1)(b.ctypes.data), None, threads))
        return {"AdvEngineID": Column(col.Int16, b)}
    if cfg == 3:
        b = np.zeros(rows, np.int64)
        _check(L.orc_datagen(3, seed, start, rows, (C.c_void_p * 1)(b.ctypes.data), None, threads))
        return {"UserID": Column(col.Int64, b)}
    if cfg == 4:
        bufs = [np.zeros(rows, np.int64), np.zeros(rows, np.int32), np.zeros(rows, np.int16), np.zeros(rows, np.int16)]
        ptrs = (C.c_void_p * 4)(*[b.ctypes.data for b in bufs])
        _check(L.orc_datagen(4, seed, start, rows, ptrs, None, threads))
        return {"WatchID": Column(col.Int64, bufs[0]), "ClientIP": Column(col.Int32, bufs[1]),
                "IsRefresh": Column(col.Int16, bufs[2]), "ResolutionWidth": Column(col.Int16, bufs[3])}
    if cfg == 5:
        cdf = c5_cdf()
        lens = np.zeros(rows, np.uint32)
        _check(L.orc_datagen(5, seed, start, rows, (C.c_void_p * 1)(lens.ctypes.data), cdf.ctypes.data, threads))
        offs = np.zeros(rows + 1, np.uint64)
        offs[1:] = np.cumsum(lens, dtype=np.uint64)
        data = np.zeros(max(1, int(offs[-1])), np.uint8)
        _check(L.orc_datagen_c5_bytes(seed, start, rows, offs.ctypes.data, data.ctypes.data, cdf.ctypes.data, threads))
        return {"SearchPhrase": Column(col.String, data[:int(offs[-1])], offs)}
    raise ValueError(cfg)


def sort_limit_indices(col: Column, asc: bool, nulls_first: bool, limit) -> np.ndarray:
    """DataBlock::sort with one column (EXP/kernels/sort.rs:79-107) -> arrow sort_to_indices ->
    indices_sorted_unstable_by (src/common/arrow/src/arrow/compute/sort/common.rs:95-174):
    NULL rows first/last in ascending row order; valid rows by ord::total_cmp / total_cmp_f32|f64
    (array/ord.rs:36-56), reversed for DESC; equal values in ascending row order (one of the
    orders select_nth_unstable_by may produce)."""
    n = len(col)
    k = n if limit is None else min(int(limit), n)
    t = col.dtype.type_id
    v = np.asarray(col.data)
    if t == abi.FLOAT64:
        b = v.astype(np.float64).view(np.uint64)
        key = np.where(b >> np.uint64(63) != 0, ~b, b | np.uint64(1 << 63))
    elif t == abi.FLOAT32:
        b = v.astype(np.float32).view(np.uint32).astype(np.uint64)
        key = np.where(b >> np.uint64(31) != 0, (~b) & np.uint64(0xFFFFFFFF), b | np.uint64(0x80000000))
    elif t in (abi.UINT8, abi.UINT16, abi.UINT32, abi.UINT64, abi.BOOLEAN):
        key = v.astype(np.uint64)
    else:
        key = v.astype(np.int64).view(np.uint64) ^ np.uint64(1 << 63)
    if not asc:
        key = ~key
    valid = np.ones(n, dtype=bool) if col.validity is None or not col.dtype.nullable else np.asarray(col.validity, bool)
    rows = np.arange(n, dtype=np.int64)
    nulls = rows[~valid]
    vrows = rows[valid]
    vsorted = vrows[np.argsort(key[valid], kind="stable")]
    order = np.concatenate([nulls, vsorted]) if nulls_first else np.concatenate([vsorted, nulls])
    return order[:k]


def _order_rank(col: Column) -> np.ndarray:
    """Per-row rank of the value in the column's ascending value order (equal values, equal rank):
    ord::total_cmp for integers, IEEE totalOrder for floats (array/ord.rs:36-56), i128 order for
    Decimal128, byte-wise (then shorter first) for strings."""
    t = col.dtype.type_id
    n = len(col)
    if t == abi.STRING:
        o = np.asarray(col.offsets, np.int64)
        d = bytes(np.asarray(col.data, np.uint8))
        vals = np.empty(n, dtype=object)
        for i in range(n):
            vals[i] = d[o[i]:o[i + 1]]
    elif t == abi.DECIMAL128:
        raw = bytes(np.asarray(col.data, np.uint8))
        vals = np.empty(n, dtype=object)
        for i in range(n):
            vals[i] = int.from_bytes(raw[16 * i:16 * i + 16], "little", signed=True)
    else:
        v = np.asarray(col.data)
        if t == abi.FLOAT64:
            b = v.astype(np.float64).view(np.uint64)
            vals = np.where(b >> np.uint64(63) != 0, ~b, b | np.uint64(1 << 63))
        elif t == abi.FLOAT32:
            b = v.astype(np.float32).view(np.uint32).astype(np.uint64)
            vals = np.where(b >> np.uint64(31) != 0, (~b) & np.uint64(0xFFFFFFFF), b | np.uint64(0x80000000))
        elif t in (abi.UINT8, abi.UINT16, abi.UINT32, abi.UINT64, abi.BOOLEAN):
            vals = v.astype(np.uint64)
        else:
            vals = v.astype(np.int64)
    _, inv = np.unique(vals, return_inverse=True)
    return inv.astype(np.int64).reshape(-1)


def sort_multi_limit_indices(cols: Sequence[Column], asc: Sequence[bool], nulls_first: Sequence[bool], limit) -> np.ndarray:
    """DataBlock::sort with several descriptions (EXP/kernels/sort.rs:79-107) -> arrow
    lexsort_to_indices: rows compare column by column — NULLs first or last per the column's
    nulls_first, values in the column's order reversed for DESC (NULL placement is not reversed);
    rows equal on every column in ascending row order (one of the orders the reference's
    unstable sort may produce)."""
    n = len(cols[0])
    k = n if limit is None else min(int(limit), n)
    keys = [np.arange(n, dtype=np.int64)]  # least significant: row index
    for c, a, nf in reversed(list(zip(cols, asc, nulls_first))):
        valid = np.ones(n, bool) if c.validity is None or not c.dtype.nullable else np.asarray(c.validity, bool)
        rank = _order_rank(c)
        rank = np.where(valid, rank if a else -rank, 0)
        null_rank = np.where(valid, 1 if nf else 0, 0 if nf else 1)
        keys.append(rank)
        keys.append(null_rank)
    return np.lexsort(keys)[:k]
