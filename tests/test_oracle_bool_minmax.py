"""The oracle's Boolean MIN / MAX (MinMaxAnyState<BooleanType>, FUN/aggregate_min_max_any.rs:
116-150) against a Python restatement: MIN = false if any non-NULL false, MAX = true if any
non-NULL true, NULL when the group has no non-NULL value (OrNull); result type Boolean."""
import numpy as np

from databend_amd import abi
from databend_amd import column as col
from databend_amd.column import Column
from tests.test_gpu_parity import oracle_aggregate


def test_oracle_bool_min_max():
    rng = np.random.default_rng(3)
    n = 5000
    g = rng.integers(0, 40, n)
    vals = rng.random(n) < 0.9
    valid = (rng.random(n) < 0.7) & (g != 11)
    k = Column.from_numbers(col.Int32, g)
    b = Column.from_bools(vals, validity=valid)
    ok, oa = oracle_aggregate([k], [("min", b), ("max", b)])
    assert oa[0].dtype.type_id == abi.BOOLEAN and oa[0].dtype.nullable
    mins, maxs = oa[0].values(), oa[1].values()
    for i, key in enumerate(ok[0].data):
        sel = (g == key) & valid
        if not sel.any():
            assert mins[i] is None and maxs[i] is None
        else:
            assert bool(mins[i]) == bool(vals[sel].all()) and bool(maxs[i]) == bool(vals[sel].any())
