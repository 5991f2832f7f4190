"""COUNT(DISTINCT x) GROUP BY keys on the GPU table.

The reference builds `count(DISTINCT x)` as AggregateDistinctCombinator over count
(FUN/aggregate_combinator_distinct.rs:60-140, 186-240): a per-group set of the argument values,
merge_result = the set's size as UInt64; a nullable argument is first stripped by the Null
combinator, so NULLs are not counted (FUN/aggregate_function_factory.rs:188-211).  ClickBench
Q9/Q14 (`SELECT RegionID, COUNT(DISTINCT UserID) … GROUP BY RegionID`) are this shape.

On the GPU the per-group set is itself a GROUP BY: phase 1 aggregates (keys…, x) WHERE
x IS NOT NULL [AND the query's predicate] into distinct pairs, phase 2 counts the pairs per key —
two passes of the same HBM table, no per-group set objects.
"""
from __future__ import annotations

from typing import Optional, Sequence

from . import abi
from .aggregates import AggregateFunctionFactory
from .aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from .column import Column, DataBlock
from .filter import FilterProgram, Pred, and_, is_not_null


def count_distinct(group_columns: Sequence[Column], arg: Column, filter_pred: Optional[Pred] = None,
                   filter_columns: Sequence[Column] = ()) -> DataBlock:
    """[count_distinct UInt64, group columns…] (TransformFinalAggregate's column order)."""
    F = AggregateFunctionFactory.instance()
    keys = list(group_columns)
    rows = len(keys[0]) if keys else len(arg)
    fcols = [c.to_abi() for c in filter_columns]
    pred = filter_pred
    if arg.dtype.nullable:
        cond = is_not_null(len(fcols))
        fcols.append(arg.to_abi())
        pred = cond if pred is None else and_(pred, cond)
    prog = FilterProgram(pred, fcols) if pred is not None else None
    # phase 1: the distinct (keys…, x) pairs
    p1 = AggregatorParams([k.dtype for k in keys] + [arg.dtype], [F.get("count")])
    t1 = AggregateHashTable(p1, HashTableConfig(True))
    try:
        t1.add_groups(keys + [arg], [None], rows=rows, filter_program=prog)
        pairs = t1.merge_result()
    finally:
        t1.close()
    pair_keys = pairs.columns[1:1 + len(keys)]
    # phase 2: pairs per key
    p2 = AggregatorParams([k.dtype for k in keys], [F.get("count")])
    t2 = AggregateHashTable(p2, HashTableConfig(False))
    try:
        n = pairs.num_rows()
        if n:
            t2.add_groups(pair_keys, [None], rows=n)
        out = t2.merge_result()
    finally:
        t2.close()
    return out
