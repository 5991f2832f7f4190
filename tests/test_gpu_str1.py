"""The key-caching insert for one non-null String key (agg.hip agg_insert_str1_kernel, ClickBench
Q13's shape: SELECT SearchPhrase, COUNT(*) ... WHERE SearchPhrase <> '' GROUP BY SearchPhrase)
against the oracle.  It runs once the table is larger than the short-key insert takes (> 65536
slots), so every case here has tens of thousands of groups or a large capacity hint: keys of 0-48
bytes (the 32-byte cache boundary and keys past it, which compare against the representative
row), a skewed key frequency (LDS hits, LDS flushes, HBM misses), several batches (later batches
find slots claimed by earlier ones), table growth (the rehash carries the cache), host and device
inputs, no predicate and `<> ''` / `= ''`, and aggregates beside COUNT(*)."""
import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.column import Column
from databend_amd.filter import cmp
from tests.parity import assert_results_equal
from tests.test_gpu_parity import gpu_aggregate, oracle_aggregate

pytestmark = pytest.mark.gpu


def _phrases(rng, n_distinct, n, lens=(0, 49), zipf=1.1):
    lo, hi = lens
    words = set()
    while len(words) < n_distinct:
        ln = int(rng.integers(lo, hi))
        words.add(bytes(rng.integers(32, 127, ln, dtype=np.uint8)))
    words = sorted(words)
    if zipf:  # bounded Zipf(s) over the distinct keys
        w = 1.0 / np.arange(1, n_distinct + 1) ** zipf
        ranks = rng.choice(n_distinct, n, p=w / w.sum())
    else:
        ranks = rng.integers(0, n_distinct, n)
    perm = rng.permutation(n_distinct)  # hot keys of every length
    return Column.from_strings([words[perm[r]] for r in ranks])


def _check(keys, aggs, filt=None, **kw):
    gk, ga = gpu_aggregate(keys, aggs, filt, **kw)
    ok, oa = oracle_aggregate(keys, aggs, filt)
    assert_results_equal(gk, ga, ok, oa)
    return len(gk[0]) if gk else 0


@pytest.mark.parametrize("on_device", [False, True])
@pytest.mark.parametrize("pred", [None, "<>", "="])
def test_str1_zipf_count(on_device, pred):
    rng = np.random.default_rng(11 + (pred == "<>") + 2 * (pred == "="))
    n = 600_000
    k = _phrases(rng, 120_000, n)
    filt = (cmp(0, pred, ""), [k]) if pred else None
    g = _check([k], [("count", None)], filt, on_device=on_device, batches=3)
    assert pred == "=" or g > 45_000


@pytest.mark.parametrize("on_device", [False, True])
def test_str1_all_functions(on_device):
    rng = np.random.default_rng(5)
    n = 400_000
    k = _phrases(rng, 90_000, n, zipf=None)
    i64 = Column.from_numbers(col.Int64, rng.integers(-2**40, 2**40, n))
    i64n = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n), validity=rng.random(n) > 0.4)
    f64 = Column.from_numbers(col.Float64, rng.random(n) * 100)
    dec = Column.from_decimals(15, 2, [int(v) for v in rng.integers(-10**12, 10**12, n)])
    aggs = [("count", None), ("count", i64n), ("sum", i64), ("sum", i64n), ("avg", f64), ("min", i64n), ("max", i64),
            ("sum", dec), ("sql_avg", dec), ("max", dec)]
    _check([k], aggs, (cmp(0, "<>", ""), [k]), on_device=on_device, batches=2)


@pytest.mark.parametrize("lens", [(33, 80), (31, 34), (0, 3)])
def test_str1_key_lengths(lens):
    """keys past the cache (compared against the representative row), at its boundary, and tiny
    keys (many of them the empty string) — with no predicate, so '' is a group of its own."""
    rng = np.random.default_rng(lens[0] * 7 + lens[1])
    n = 500_000
    nd = 80_000 if lens[1] > 3 else 95**2 + 95 + 1
    k = _phrases(rng, min(nd, 80_000), n, lens=lens, zipf=1.05)
    g = _check([k], [("count", None)], on_device=True, batches=2, capacity_hint=1 << 17)
    assert g > 5_000


def test_str1_big_table_few_groups():
    """a capacity hint sizes the table far beyond the groups: the key-caching insert runs with a
    few hot groups that every workgroup flushes into the same HBM slots."""
    rng = np.random.default_rng(3)
    n = 300_000
    k = _phrases(rng, 40, n, lens=(1, 40), zipf=None)
    g = _check([k], [("count", None), ("sum", Column.from_numbers(col.Int64, rng.integers(0, 100, n)))],
               on_device=True, capacity_hint=1 << 20)
    assert g == 40


def test_str1_growth():
    """the first batch sizes the table for few groups, later batches bring many more: overflow
    growth rehashes the key-caching slots, cache words included."""
    rng = np.random.default_rng(9)
    few = _phrases(rng, 30, 200_000, zipf=None)
    many = _phrases(rng, 200_000, 600_000, zipf=None)
    k = Column.from_strings(list(few.values()) + list(many.values()))
    g = _check([k], [("count", None)], on_device=True, batches=4, capacity_hint=70_000)
    assert g > 150_000
