"""Helpers shared by the parity tests: canonical, order-insensitive result comparison.

The reference compares GROUP BY outputs with `assert_block_value_sort_eq` (group order is not part
of the contract), so results are compared as multisets of rows.  Integer/Decimal/count/string
results must match bit for bit; float64 SUM/AVG within the north-star tolerance (rel 1e-12).
"""
import math
from typing import List, Sequence

from databend_amd import abi

FLOAT_REL_TOL = 1e-12  # BASELINE.json north_star: float64 SUM/AVG within 1e-12 relative


def rows_of(keys, aggs) -> List[tuple]:
    cols = [c.values() for c in list(keys) + list(aggs)]
    n = len(cols[0]) if cols else 0
    return [tuple(c[i] for c in cols) for i in range(n)]


def _sort_key(row):
    out = []
    for v in row:
        if v is None:
            out.append((0, 0))
        elif isinstance(v, float):
            out.append((1, (1, 0) if math.isnan(v) else (0, v)))
        else:
            out.append((1, v))
    return out


def assert_results_equal(got_keys, got_aggs, exp_keys, exp_aggs, float_rel=FLOAT_REL_TOL, n_key_cols=None):
    """Compare (keys, aggs) column lists as row multisets, sorted by the key columns."""
    g = rows_of(got_keys, got_aggs)
    e = rows_of(exp_keys, exp_aggs)
    assert len(g) == len(e), f"group count differs: got {len(g)} expected {len(e)}"
    nk = len(got_keys) if n_key_cols is None else n_key_cols
    g.sort(key=lambda r: _sort_key(r[:nk]))
    e.sort(key=lambda r: _sort_key(r[:nk]))
    for i, (a, b) in enumerate(zip(g, e)):
        for j, (x, y) in enumerate(zip(a, b)):
            if isinstance(x, float) and isinstance(y, float):
                if math.isnan(x) and math.isnan(y):
                    continue
                assert math.isclose(x, y, rel_tol=float_rel, abs_tol=0.0) or x == y, \
                    f"row {i} col {j}: {x!r} != {y!r} (rel tol {float_rel})"
            else:
                assert x == y, f"row {i} col {j}: {x!r} != {y!r}\n got row {a}\n exp row {b}"


def key_dtypes(cols) -> List[int]:
    return [c.dtype.type_id for c in cols]
