"""The vectorized result comparison (tests/parity.py _fast_compare) agrees with the row-by-row one:
same verdict on equal results in shuffled order, and it catches a changed key, count, decimal,
string or float beyond the tolerance."""
import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.column import Column
from tests import parity


def _block(rng, n):
    keys_i = rng.permutation(n).astype(np.int64) * 7 - 3
    strs = [("k%d" % (i % 977)) * (1 + i % 5) + str(i) for i in range(n)]
    ks = [Column.from_numbers(col.Int64, keys_i), Column.from_strings(strs)]
    cnt = Column.from_numbers(col.UInt64, rng.integers(1, 100, n).astype(np.uint64))
    f = Column.from_numbers(col.Float64, rng.random(n) * 1e6, validity=rng.random(n) < 0.9)
    dec = Column.from_decimals(38, 2, [int(x) * (10**20 if i % 3 == 0 else 1) for i, x in enumerate(rng.integers(-10**9, 10**9, n))])
    return ks, [cnt, f, dec]


def _take(c: Column, idx):
    if c.dtype.type_id == col.abi.STRING:
        vals = c.values()
        return Column.from_strings([vals[i] for i in idx])
    if c.dtype.type_id == col.abi.DECIMAL128:
        return Column(c.dtype, c.data.reshape(-1, 16)[idx].reshape(-1).copy(), None,
                      None if c.validity is None else c.validity[idx])
    return Column(c.dtype, c.data[idx].copy(), None, None if c.validity is None else c.validity[idx])


@pytest.mark.parametrize("n", [parity.FAST_MIN_ROWS + 17])
def test_fast_compare_matches_slow(n):
    rng = np.random.default_rng(5)
    ks, ags = _block(rng, n)
    perm = rng.permutation(n)
    ks2, ags2 = [_take(c, perm) for c in ks], [_take(c, perm) for c in ags]
    assert parity._fast_compare(ks, ags, ks2, ags2, parity.FLOAT_REL_TOL)
    parity.assert_results_equal(ks, ags, ks2, ags2)

    # a float within tolerance passes, beyond it fails
    f = ags2[1]
    f.data = f.data.copy()
    f.data[0] *= 1 + 1e-14
    parity.assert_results_equal(ks, ags, ks2, ags2)
    f.data[0] *= 1 + 1e-9
    if f.validity[0]:
        with pytest.raises(AssertionError):
            parity.assert_results_equal(ks, ags, ks2, ags2)
    f.data[0] = ags[1].data[perm[0]]

    for mutate in ("key", "str", "count", "dec"):
        k3, a3 = [_take(c, np.arange(n)) for c in ks2], [_take(c, np.arange(n)) for c in ags2]
        if mutate == "key":
            k3[0].data[5] += 1
        elif mutate == "str":
            vals = k3[1].values()
            vals[9] = vals[9] + b"x"
            k3[1] = Column.from_strings(vals)
        elif mutate == "count":
            a3[0].data[11] += 1
        else:
            a3[2].data[16 * 13 + 15] ^= 1
        with pytest.raises(AssertionError):
            parity.assert_results_equal(ks, ags, k3, a3)
