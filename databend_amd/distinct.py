"""Aggregates with the DISTINCT combinator on the GPU table.

The reference builds `f(DISTINCT x)` (`count_distinct`, `sum_distinct`, ...) as
AggregateDistinctCombinator over the nested f (FUN/aggregate_combinator_distinct.rs:60-140,
186-260): a per-group set of the argument values; merge_result feeds the set to f (count: the
set's size).  A nullable argument is stripped by the Null combinator first, so NULL is never in
the set, and the group still appears (count 0 / NULL for sum) when all its values are NULL
(FUN/aggregate_function_factory.rs:170-211).  ClickBench Q10 mixes it with plain aggregates:
`SELECT RegionID, SUM(AdvEngineID), COUNT(*), AVG(ResolutionWidth), COUNT(DISTINCT UserID)
 FROM hits GROUP BY RegionID` (benchmark/clickbench/hits/queries/09.sql).

On the GPU the per-group set is itself a GROUP BY, and every aggregate of the query lands in ONE
final table T whose aggregates take nullable arguments:

* raw rows (the query's filter fused) go into T with their plain aggregates' arguments and an
  all-NULL column for each distinct aggregate (the rows create their groups, count nothing);
* per distinct aggregate j, the rows go into a pair table P_j keyed (keys..., x_j) — NULL x_j is
  a pair of its own — whose result columns stay in HBM; its pairs then go into T with x_j as the
  argument of aggregate j and all-NULL columns for every other aggregate.  f over distinct pairs
  is f over the group's value set; NULL x_j is skipped by the nullable-argument state.

Declaring the plain aggregates' arguments nullable does not change them: every raw row is valid,
and every result that can be NULL is already Nullable through the OrNull adaptor (count stays
UInt64, count(*) becomes count of a never-NULL dummy).  Between the phases only group counts reach
the host; the pairs never leave the device.

Inside the processors (TransformPartialAggregate / TransformPartitionBucket /
TransformFinalAggregate, aggregator.py) the same split crosses the stages: the partial keeps T and
one pair table per distinct aggregate (`DistinctPartial`), at the max radix bits the reference
forces for DISTINCT (AGG/transform_aggregate_partial.rs:146-155); on_finish exports T's buckets
and each pair table's buckets bucketed by the group keys alone (dbg_agg_set_partition_keys), so a
bucket's pairs are exactly its groups' value sets — the combinator's state — and travel with it
(AggregateMeta.distinct).  The final stage (`final_distinct`) merges T's records, dedupes each
pair set across partials in a final pair table, and feeds the pairs into T as above.
"""
from __future__ import annotations

from dataclasses import replace
from typing import List, Optional, Sequence

import numpy as np

from . import abi
from .aggregates import AggregateFunction, AggregateFunctionFactory
from .aggregator import AggregateHashTable, AggregateMeta, AggregatorParams, HashTableConfig, export_buckets
from .column import Column, DataBlock, DataType
from .ffi import Unsupported

_DUMMY = DataType(abi.UINT8, 0, 0, True)  # count(*)'s never-NULL stand-in argument


def _torch():
    import torch
    return torch


class _NullSource:
    """All-NULL argument columns of any type and length: one zeroed buffer serves as data,
    offsets (strings) and the validity bitmap."""

    def __init__(self, rows: int, on_device: bool):
        nbytes = max(64, rows * 16 + 16)
        if on_device:
            self.buf = _torch().zeros(nbytes, dtype=_torch().uint8, device="cuda")
            self.ptr = self.buf.data_ptr()
        else:
            self.buf = np.zeros(nbytes, np.uint8)
            self.ptr = self.buf.ctypes.data
        self.rows = rows

    def column(self, dtype: DataType, rows: int) -> abi.dbg_column:
        assert rows <= self.rows
        c = abi.dbg_column()
        c.dt = dtype.wrap_nullable().to_abi()
        c.data = self.ptr
        c.offsets = self.ptr if dtype.type_id == abi.STRING else None
        c.validity = self.ptr
        c.len = rows
        return c


class _Ones:
    """A never-NULL UInt8 column of `rows` rows (count(*)'s dummy argument)."""

    def __init__(self, rows: int, on_device: bool):
        if on_device:
            self.buf = _torch().ones(max(1, rows), dtype=_torch().uint8, device="cuda")
            self.ptr = self.buf.data_ptr()
        else:
            self.buf = np.ones(max(1, rows), np.uint8)
            self.ptr = self.buf.ctypes.data

    def column(self, rows: int) -> abi.dbg_column:
        c = abi.dbg_column()
        c.dt = _DUMMY.to_abi()
        c.data = self.ptr
        c.len = rows
        return c


def _check_supported(keys: Sequence[DataType], functions: Sequence[AggregateFunction]) -> None:
    if not keys:
        raise Unsupported(abi.DBG_ERR_UNSUPPORTED, "DISTINCT aggregates without GROUP BY keys run in the "
                          "reference's single-key processor (AGG/transform_single_key.rs), not on this path")
    for f in functions:
        if f.distinct and f.arg is None:
            raise Unsupported(abi.DBG_ERR_UNSUPPORTED, f"{f.display_name}: DISTINCT needs an argument")
        if f.distinct and f.arg.type_id == abi.BOOLEAN:
            raise Unsupported(abi.DBG_ERR_UNSUPPORTED, "DISTINCT over Boolean stays on the CPU path")
    if any(t.type_id == abi.BOOLEAN for t in keys):
        raise Unsupported(abi.DBG_ERR_UNSUPPORTED, "Boolean group keys with DISTINCT stay on the CPU path")
    for f in functions:
        # the final table declares every plain aggregate's argument nullable; that keeps the result
        # type only when the function already returns Nullable (the OrNull adaptor, the factory's
        # default) or cannot return NULL at all (count)
        if not f.distinct and not f.or_null and f.arg is not None and f.kind != abi.AGG_COUNT:
            raise Unsupported(abi.DBG_ERR_UNSUPPORTED, f"{f.display_name}: a non-OrNull {f.name()} beside DISTINCT "
                              "would change its result type; it stays on the CPU path")


class DistinctAggregator:
    """One GROUP BY whose aggregate list may hold DISTINCT aggregates (AggregatorParams with
    `AggregateFunction.distinct`), run as described in the module docstring.  `run` returns the
    TransformFinalAggregate block [agg results..., group columns...]."""

    def __init__(self, params: AggregatorParams, device: int = -1):
        self.params = params
        self.device = device
        _check_supported(params.group_data_types, params.aggregate_functions)
        fns = []
        for f in params.aggregate_functions:
            if f.arg is None:
                fns.append(replace(f, arg=_DUMMY, distinct=False))
            else:
                fns.append(replace(f, arg=f.arg.wrap_nullable(), distinct=False))
        self.t_params = AggregatorParams(list(params.group_data_types), fns)
        self.distinct_idx = [j for j, f in enumerate(params.aggregate_functions) if f.distinct]

    def run(self, group_columns: Sequence, args: Sequence, filter_program=None,
            rows: Optional[int] = None, on_device: Optional[bool] = None) -> DataBlock:
        """group_columns / args (one per aggregate, None for count(*)): host Columns or
        DeviceColumns, like AggregateHashTable.add_groups."""
        if rows is None:
            rows = len(group_columns[0])
        if on_device is None:
            on_device = not isinstance(group_columns[0], Column)
        fns = self.params.aggregate_functions
        keys = [c.to_abi() for c in group_columns]
        nulls = _NullSource(rows, on_device)
        ones = _Ones(rows, on_device)
        keep = [nulls, ones]
        final = AggregateHashTable(self.t_params, HashTableConfig(False), self.device)
        try:
            # raw rows: plain aggregates' arguments, all-NULL for the distinct ones
            a = []
            for j, f in enumerate(fns):
                if f.distinct:
                    a.append(nulls.column(f.arg, rows))
                elif args[j] is None:
                    a.append(ones.column(rows))
                else:
                    a.append(args[j].to_abi())
            final.add_groups_abi(keys, a, rows, filter_program, on_device)
            # each distinct aggregate: pairs (keys..., x) in HBM, then into the final table
            for j in self.distinct_idx:
                pairs = self._pairs(group_columns, args[j], filter_program, rows, on_device)
                keep.append(pairs)
                n = len(pairs[0])
                if n == 0:
                    continue
                big = nulls if (on_device and n <= rows) else _NullSource(n, True)  # pairs live in HBM
                keep.append(big)
                a = []
                for i, f in enumerate(fns):
                    if i == j:
                        a.append(pairs[-1].to_abi())
                    else:
                        a.append(big.column(_DUMMY if f.arg is None else f.arg, n))
                final.add_groups_abi([c.to_abi() for c in pairs[:-1]], a, n, None, True)
            return final.merge_result()
        finally:
            final.close()

    def _pairs(self, group_columns, x, filter_program, rows, on_device):
        """P_j: the distinct (keys..., x) of the selected rows, as device columns."""
        F = AggregateFunctionFactory.instance()
        xt = x.dtype
        p = AggregatorParams(list(self.params.group_data_types) + [xt], [F.get("count")])
        t = AggregateHashTable(p, HashTableConfig(True), self.device)
        try:
            t.add_groups(list(group_columns) + [x], [None], rows=rows, filter_program=filter_program,
                         on_device=on_device)
            out = t.merge_result_device()
        finally:
            t.close()
        return out[1:]  # drop the pair count: [keys..., x]


def count_distinct(group_columns: Sequence[Column], arg: Column, filter_pred=None,
                   filter_columns: Sequence[Column] = ()) -> DataBlock:
    """[count_distinct(arg) UInt64, group columns...] — the lone COUNT(DISTINCT x) GROUP BY keys
    shape of ClickBench Q9/Q14."""
    from .filter import FilterProgram
    F = AggregateFunctionFactory.instance()
    keys = list(group_columns)
    params = AggregatorParams([k.dtype for k in keys], [F.get("count_distinct", [], [arg.dtype])])
    prog = FilterProgram(filter_pred, list(filter_columns)) if filter_pred is not None else None
    return DistinctAggregator(params).run(keys, [arg], filter_program=prog)


# ---- the processor form (aggregator.py): pair sets crossing the partial -> final boundary ----

def _t_params(params: AggregatorParams) -> AggregatorParams:
    fns = []
    for f in params.aggregate_functions:
        if f.arg is None:
            fns.append(replace(f, arg=_DUMMY, distinct=False))
        else:
            fns.append(replace(f, arg=f.arg.wrap_nullable(), distinct=False))
    return AggregatorParams(list(params.group_data_types), fns)


def _pair_params(params: AggregatorParams, j: int) -> AggregatorParams:
    F = AggregateFunctionFactory.instance()
    return AggregatorParams(list(params.group_data_types) + [params.aggregate_functions[j].arg], [F.get("count")])


def _pair_table(params: AggregatorParams, j: int, partial: bool, device: int) -> AggregateHashTable:
    t = AggregateHashTable(_pair_params(params, j), HashTableConfig(partial), device)
    t.set_strategy(abi.STRATEGY_TABLE)  # bucketing by the key prefix is a table-strategy export
    t.set_partition_keys(len(params.group_data_types))
    return t


class DistinctPartial:
    """TransformPartialAggregate's state for a query with DISTINCT aggregates: the main table T
    (plain aggregates; the distinct ones' arguments NULL) and one pair table per distinct
    aggregate, all fed from the same blocks."""

    def __init__(self, params: AggregatorParams, device: int = -1):
        _check_supported(params.group_data_types, params.aggregate_functions)
        self.params = params
        self.device = device
        self.t_params = _t_params(params)
        self.table = AggregateHashTable(self.t_params, HashTableConfig(True), device)
        self.distinct_idx = [j for j, f in enumerate(params.aggregate_functions) if f.distinct]
        self.pairs = {j: _pair_table(params, j, True, device) for j in self.distinct_idx}
        self._keep = []

    def add_groups(self, group_columns, args, rows: int, filter_program=None) -> None:
        on_device = not isinstance(group_columns[0], Column)
        fns = self.params.aggregate_functions
        nulls = _NullSource(rows, on_device)
        ones = _Ones(rows, on_device)
        a = []
        for j, f in enumerate(fns):
            if f.distinct:
                a.append(nulls.column(f.arg, rows))
            elif args[j] is None:
                a.append(ones.column(rows))
            else:
                a.append(args[j].to_abi())
        self.table.add_groups_abi([c.to_abi() for c in group_columns], a, rows, filter_program, on_device)
        for j in self.distinct_idx:
            self.pairs[j].add_groups(list(group_columns) + [args[j]], [None], rows=rows, filter_program=filter_program,
                                     on_device=on_device)
        if on_device:  # the device inputs of the staged launches must outlive them
            self._keep.append((nulls, ones))

    def retained_bytes(self) -> int:
        """Device bytes the main table and the pair tables keep for the inputs they reference."""
        return self.table.retained_bytes() + sum(t.retained_bytes() for t in self.pairs.values())

    def compact(self) -> None:
        """dbg_agg_compact of the main table and every pair table: each then references one record
        batch of its own groups (or pairs), so the copies of earlier host blocks are released and
        the partial's memory follows its groups and value sets, not the rows it saw.  Compaction
        synchronises the table's stream, so the device columns kept for staged launches are free
        to go too — but only when every table compacted: dbg_agg_compact returns early (no
        synchronisation) for inline-key or partitioned handles, whose staged launches may still
        read the kept columns."""
        done = self.table.compact()
        for t in self.pairs.values():
            done = t.compact() and done
        if done:
            self._keep.clear()

    def on_finish(self, n_parts: int) -> List[AggregateMeta]:
        t_b = export_buckets(self.table, n_parts)
        p_b = {j: export_buckets(self.pairs[j], n_parts) for j in self.distinct_idx}
        out = []
        for b in range(n_parts):
            d = [p_b[j][b] for j in self.distinct_idx]
            if len(t_b[b]) or any(len(x) for x in d):
                out.append(AggregateMeta(b, t_b[b], n_parts, distinct=d))
        return out

    def close(self):
        self.table.close()
        for t in self.pairs.values():
            t.close()
        self._keep.clear()


def repartition_distinct(params: AggregatorParams, meta: AggregateMeta, n_parts: int, device: int = -1) -> List[AggregateMeta]:
    """TransformPartitionBucket's alignment of a DISTINCT meta written with fewer buckets: T's
    payload and every pair payload re-exported at n_parts buckets (pairs by their group keys)."""
    import torch
    t_params = _t_params(params)
    idx = [j for j, f in enumerate(params.aggregate_functions) if f.distinct]
    scratch = AggregateHashTable(t_params, HashTableConfig(True), device)
    pts = {j: _pair_table(params, j, True, device) for j in idx}
    try:
        p = meta.payload
        if p is not None and len(p):
            scratch.merge_records(p.records, p.strings, [p.n_records], [p.string_bytes])
        for j, q in zip(idx, meta.distinct):
            if len(q):
                pts[j].merge_records(q.records, q.strings, [q.n_records], [q.string_bytes])
        t_b = export_buckets(scratch, n_parts)
        p_b = {j: export_buckets(pts[j], n_parts) for j in idx}
        torch.cuda.current_stream().synchronize()
    finally:
        scratch.close()
        for t in pts.values():
            t.close()
    out = []
    for b in range(n_parts):
        d = [p_b[j][b] for j in idx]
        if len(t_b[b]) or any(len(x) for x in d):
            out.append(AggregateMeta(b, t_b[b], n_parts, distinct=d))
    return out


def final_distinct(params: AggregatorParams, items: Sequence[AggregateMeta], device: int = -1) -> DataBlock:
    """TransformFinalAggregate for one bucket of a query with DISTINCT aggregates: T merges every
    partial's states; each distinct aggregate's pairs are deduplicated across partials in a final
    pair table, then enter T as that aggregate's argument (the other aggregates' arguments NULL)."""
    if any(m.is_serialized() for m in items):
        raise Unsupported(abi.DBG_ERR_UNSUPPORTED, "serialized DISTINCT states (borsh sets) stay on the CPU final")
    t_params = _t_params(params)
    fns = params.aggregate_functions
    idx = [j for j, f in enumerate(fns) if f.distinct]
    if not any((m.payload is not None and len(m.payload)) or any(len(x) for x in (m.distinct or [])) for m in items):
        return params.empty_result_block()
    final = AggregateHashTable(t_params, HashTableConfig(False), device)
    keep = []
    try:
        for m in items:
            p = m.payload
            if p is not None and len(p):
                final.merge_records(p.records, p.strings, [p.n_records], [p.string_bytes])
        for jj, j in enumerate(idx):
            pt = _pair_table(params, j, False, device)
            try:
                for m in items:
                    q = m.distinct[jj]
                    if len(q):
                        pt.merge_records(q.records, q.strings, [q.n_records], [q.string_bytes])
                pairs = pt.merge_result_device()[1:]  # [keys..., x]
            finally:
                pt.close()
            keep.append(pairs)
            n = len(pairs[0])
            if n == 0:
                continue
            nulls = _NullSource(n, True)
            keep.append(nulls)
            a = []
            for i, f in enumerate(fns):
                if i == j:
                    a.append(pairs[-1].to_abi())
                else:
                    a.append(nulls.column(_DUMMY if f.arg is None else f.arg, n))
            final.add_groups_abi([c.to_abi() for c in pairs[:-1]], a, n, None, True)
        return final.merge_result()
    finally:
        final.close()
