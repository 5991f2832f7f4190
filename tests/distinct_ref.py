"""Pure-Python restatement of AggregateDistinctCombinator for small inputs (TEST INFRASTRUCTURE).

FUN/aggregate_combinator_distinct.rs:60-140: per group, the SET of non-NULL argument values (the
Null combinator strips NULLs first, FUN/aggregate_function_factory.rs:170-211); merge_result runs
the nested function over the set (count: its size, UInt64, never NULL; sum/min/max/avg: NULL when
the set is empty — the OrNull / Null adaptors).  Pinned by the reference's sum_distinct goldens
(tests/golden/distinct_goldens.json, transcribed from agg_group_by.txt / agg.txt by
make_golden.py) and 03_0022_select_distinct.test:21-24.
"""
from decimal import Decimal, ROUND_DOWN


def distinct_aggregate(keys, fn, values, valid=None):
    """keys: list of hashable group keys; values: python values; valid: bools or None.
    Returns {key: result} with None for a NULL result.  Sums of ints wrap like the release build
    only beyond 64 bits, which these small tests never reach."""
    sets = {}
    for i, k in enumerate(keys):
        s = sets.setdefault(k, set())
        if valid is None or valid[i]:
            s.add(values[i])
    out = {}
    for k, s in sets.items():
        if fn == "count":
            out[k] = len(s)
        elif not s:
            out[k] = None
        elif fn == "sum":
            out[k] = sum(s)
        elif fn == "min":
            out[k] = min(s)
        elif fn == "max":
            out[k] = max(s)
        elif fn == "avg":  # numbers: sum as f64 / count as f64 (aggregate_avg.rs:90-98)
            out[k] = float(sum(s)) / float(len(s))
        else:
            raise ValueError(fn)
    return out


def decimal_avg(total: int, count: int, scale_add: int) -> int:
    """DecimalAvgState: value * 10^scale_add, truncating division (aggregate_avg.rs:173-201)."""
    q = Decimal(total * 10 ** scale_add) / Decimal(count)
    return int(q.to_integral_value(rounding=ROUND_DOWN))
