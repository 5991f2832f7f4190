"""The short-key specialisation of the generic insert (agg.hip agg_insert_short_kernel: one or two
non-null String keys packed with their length into a word per key, compared in LDS; COUNT / SUM /
AVG over non-nullable arguments loaded with the row) against the oracle: TPC-H Q1's shape,
keys of every length 0..12 (those over 7 bytes take the generic path inside the same launch),
more groups than one LDS table holds (the full-table fallback), the empty string, a filter, host
and device inputs, and several batches."""
import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.column import Column
from databend_amd.filter import cmp
from tests.test_gpu_parity import check_parity

pytestmark = pytest.mark.gpu


def _strings(rng, n, pool):
    return Column.from_strings([pool[i] for i in rng.integers(0, len(pool), n)])


@pytest.mark.parametrize("on_device", [False, True])
@pytest.mark.parametrize("case", ["q1", "lengths", "many_groups", "one_key"])
def test_short_keys_match_oracle(case, on_device):
    rng = np.random.default_rng(len(case) * 13 + on_device)
    n = 400_000
    if case == "q1":
        keys = [_strings(rng, n, [b"A", b"N", b"R"]), _strings(rng, n, [b"F", b"O"])]
    elif case == "lengths":
        pool = [b"", b"x", b"ab", b"abc", b"abcdefg", b"abcdefgh", b"0123456789ab", b"zzzzzzz", b"abcdefg\x00"]
        keys = [_strings(rng, n, pool), _strings(rng, n, pool[:5])]
    elif case == "many_groups":
        pool = [b"k%05d" % v for v in range(3000)]  # 6-byte keys, far more than one LDS table
        keys = [_strings(rng, n, pool), _strings(rng, n, [b"", b"q"])]
    else:
        keys = [_strings(rng, n, [b"p%d" % v for v in range(50)])]
    dec = Column.from_decimals(15, 2, [int(v) for v in rng.integers(-10**12, 10**12, n)])
    dec38 = Column.from_decimals(38, 6, [int(v) * 10**20 for v in rng.integers(-10**9, 10**9, n)])
    i64 = Column.from_numbers(col.Int64, rng.integers(-2**40, 2**40, n))
    i16 = Column.from_numbers(col.Int16, rng.integers(-300, 300, n))
    f64 = Column.from_numbers(col.Float64, rng.random(n) * 100)
    d = Column.from_numbers(col.Date, rng.integers(9000, 11000, n))
    aggs = [("sum", dec), ("sum", dec38), ("sql_avg", dec), ("avg", i64), ("sum", i16), ("count", None),
            ("count", i64), ("avg", f64)]
    check_parity(keys, aggs, filt=(cmp(0, "<=", 10471), [d]), on_device=on_device, batches=2)
    check_parity(keys, aggs[:3], on_device=on_device)
