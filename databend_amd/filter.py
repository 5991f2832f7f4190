"""Predicate programs for the filter stage (mirror of EXP/filter/select_expr.rs `SelectExpr`).

Databend's `SelectExprBuilder` turns the AND-reduced predicate into a tree of
`And`/`Or`/`Compare`/`Others` nodes (select_expr.rs:30-...); `Selector::select` walks it to fill a
u32 selection vector (selector.rs:64-325).  Here the same tree is flattened to a postfix program of
`dbg_pred_node`s that the HIP kernel evaluates per row with SQL three-valued logic (rows are kept
only when the predicate is TRUE, filter_executor.rs:73-128).

    pred = and_(cmp(0, "<=", 10471), not_(is_null(1)))
"""
from __future__ import annotations

import ctypes as C
from decimal import Decimal
from typing import List, Sequence

from . import abi
from .column import Column

_CMP = {"=": abi.CMP_EQ, "==": abi.CMP_EQ, "<>": abi.CMP_NE, "!=": abi.CMP_NE, "<": abi.CMP_LT,
        "<=": abi.CMP_LE, ">": abi.CMP_GT, ">=": abi.CMP_GE}


class Pred:
    def postfix(self) -> List[dict]:
        raise NotImplementedError


class _Cmp(Pred):
    def __init__(self, col: int, op: str, const):
        self.col, self.op, self.const = col, op, const

    def postfix(self):
        return [dict(op=abi.PRED_CMP_CONST, cmp=_CMP[self.op], col=self.col, const=self.const)]


class _CmpCols(Pred):
    def __init__(self, a: int, op: str, b: int):
        self.a, self.op, self.b = a, op, b

    def postfix(self):
        return [dict(op=abi.PRED_CMP_COLS, cmp=_CMP[self.op], col=self.a, col2=self.b)]


class _Bin(Pred):
    def __init__(self, op: int, a: Pred, b: Pred):
        self.op, self.a, self.b = op, a, b

    def postfix(self):
        return self.a.postfix() + self.b.postfix() + [dict(op=self.op)]


class _Un(Pred):
    def __init__(self, op: int, a: Pred = None, col: int = 0):
        self.op, self.a, self.col = op, a, col

    def postfix(self):
        if self.op == abi.PRED_NOT:
            return self.a.postfix() + [dict(op=self.op)]
        return [dict(op=self.op, col=self.col)]


def cmp(col: int, op: str, const) -> Pred:
    return _Cmp(col, op, const)


def cmp_cols(a: int, op: str, b: int) -> Pred:
    return _CmpCols(a, op, b)


def and_(*ps: Pred) -> Pred:
    out = ps[0]
    for p in ps[1:]:
        out = _Bin(abi.PRED_AND, out, p)
    return out


def or_(*ps: Pred) -> Pred:
    out = ps[0]
    for p in ps[1:]:
        out = _Bin(abi.PRED_OR, out, p)
    return out


def not_(p: Pred) -> Pred:
    return _Un(abi.PRED_NOT, p)


def is_null(col: int) -> Pred:
    return _Un(abi.PRED_IS_NULL, col=col)


def is_not_null(col: int) -> Pred:
    return _Un(abi.PRED_IS_NOT_NULL, col=col)


def true_() -> Pred:
    return _Un(abi.PRED_TRUE)


class FilterProgram:
    """A predicate bound to its columns, marshalled as `dbg_filter` (kept alive by this object).
    `cols` holds `dbg_column` structs or column objects (Column / DeviceColumn): objects are kept
    referenced here, so a device column's HBM outlives kernels still queued on it as long as the
    program does (add_groups retains the program of an on-device batch until reset/close)."""

    def __init__(self, pred: Pred, cols: Sequence):
        self.pred = pred
        self._owners = [c for c in cols if hasattr(c, "to_abi")]
        self.cols = [c.to_abi() if hasattr(c, "to_abi") else c for c in cols]
        post = pred.postfix()
        self._keep = []
        self.nodes = (abi.dbg_pred_node * len(post))()
        for i, d in enumerate(post):
            n = self.nodes[i]
            n.op = d["op"]
            n.cmp = d.get("cmp", 0)
            n.col = d.get("col", 0)
            n.col2 = d.get("col2", 0)
            if "const" in d:
                self._set_const(n, self.cols[n.col], d["const"])
        self.col_arr = (abi.dbg_column * max(1, len(self.cols)))(*self.cols)
        self.struct = abi.dbg_filter(self.nodes, len(post), len(self.cols), self.col_arr)

    def _set_const(self, n: abi.dbg_pred_node, col: abi.dbg_column, v):
        t = col.dt.type
        if t == abi.STRING:
            b = v.encode() if isinstance(v, str) else bytes(v)
            buf = C.create_string_buffer(b, max(1, len(b)))
            self._keep.append(buf)
            n.str = C.addressof(buf)
            n.str_len = len(b)
        elif t in (abi.FLOAT32, abi.FLOAT64):
            n.f64 = float(v)
        elif t == abi.DECIMAL128:
            if isinstance(v, Decimal):
                v = int(v.scaleb(col.dt.scale))
            v = int(v)
            u = v & ((1 << 128) - 1)
            n.i128_lo = u & ((1 << 64) - 1)
            hi = u >> 64
            n.i128_hi = hi - (1 << 64) if hi >= (1 << 63) else hi
        elif t in (abi.UINT8, abi.UINT16, abi.UINT32, abi.UINT64):
            u = int(v) & ((1 << 64) - 1)
            n.i64 = u - (1 << 64) if u >= (1 << 63) else u
        else:
            n.i64 = int(v)

    def ptr(self):
        return C.byref(self.struct)


class FilterExecutor:
    """FilterExecutor (EXP/filter/filter_executor.rs:73-128) over device-resident blocks:
    `select` fills the ascending u32 selection of rows where the predicate is TRUE
    (dbg_filter_select), `take` gathers every column of the block at it (DataBlock::take,
    EXP/kernels/take.rs:56-91: dbg_take_fixed / dbg_take_string), `filter` does both.  The
    GROUP BY path never materialises the filtered block: its insert evaluates the predicate itself."""

    def __init__(self, pred: Pred, predicate_columns: Sequence[int]):
        self.pred = pred
        self.predicate_columns = list(predicate_columns)

    def select(self, columns, rows: int):
        import torch
        from .ffi import check, lib
        prog = FilterProgram(self.pred, [columns[i] for i in self.predicate_columns])
        sel = torch.empty(max(1, rows), dtype=torch.int32, device=columns[0].data.device)
        n = C.c_uint64()
        check(lib().dbg_filter_select(prog.ptr(), rows, sel.data_ptr(), C.byref(n), None))
        return sel[: n.value]

    def take(self, columns, sel):
        from .sort import take
        return [take(c, sel) for c in columns]

    def filter(self, columns, rows: int):
        sel = self.select(columns, rows)
        if sel.numel() == rows:  # everything selected: the block passes through (filter_executor.rs:95-100)
            return list(columns)
        return self.take(columns, sel)
