"""CPU: the Python restatement of the DISTINCT combinator (tests/distinct_ref.py) against the
reference's own sum_distinct goldens and 03_0022_select_distinct.test:21-24, plus the host-side
factory rules for `*_distinct` names (no GPU)."""
import json
import os

import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.ffi import Unsupported
from tests.distinct_ref import distinct_aggregate

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "distinct_goldens.json")))
F = AggregateFunctionFactory.instance()


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"{c['fn']}({c['arg']})-{'gb' if c['grouped'] else 'one'}")
def test_restatement_matches_reference_goldens(case):
    inp = GOLD["inputs"][case["arg"]]
    keys = [0, 1, 0, 1] if case["grouped"] else [0, 0, 0, 0]
    got = distinct_aggregate(keys, case["fn"].replace("_distinct", ""), inp["values"], inp["validity"])
    exp = [v if ok else None for v, ok in zip(case["values"], case["validity"])]
    assert [got[k] for k in sorted(got)] == exp, case["source"]


def test_restatement_matches_slt_count_distinct():
    # SELECT count(distinct number % 3) c FROM numbers(1000) WHERE number > 3  ->  3
    vals = [n % 3 for n in range(1000) if n > 3]
    assert distinct_aggregate([0] * len(vals), "count", vals) == {0: 3}


def test_factory_distinct_suffix():
    f = F.get("count_distinct", [], [col.Int64.wrap_nullable()])
    assert f.distinct and f.kind == abi.AGG_COUNT
    assert f.return_type() == col.UInt64  # count: default on NULL-only input, never Nullable
    s = F.get("sum_distinct", [], [col.Int64])
    assert s.return_type() == col.Int64.wrap_nullable()
    with pytest.raises(Unsupported):
        s.to_abi()  # a distinct aggregate is not one table state: DistinctAggregator runs it


def test_non_or_null_plain_aggregate_beside_distinct_is_unsupported():
    """DistinctAggregator declares every plain aggregate's argument nullable in its final table;
    a sum/min/max/avg built without the OrNull adaptor would change its result type, so it is
    refused (UNSUPPORTED: the caller keeps the CPU path) — no device needed to decide."""
    import pytest
    from databend_amd import column as col
    from databend_amd.aggregates import AggregateFunctionFactory
    from databend_amd.aggregator import AggregatorParams
    from databend_amd.distinct import DistinctAggregator
    from databend_amd.ffi import Unsupported
    F = AggregateFunctionFactory.instance()
    ok = AggregatorParams([col.Int32], [F.get("count_distinct", [], [col.Int64]), F.get("sum", [], [col.Int64])])
    DistinctAggregator(ok)
    bad = AggregatorParams([col.Int32], [F.get("count_distinct", [], [col.Int64]),
                                         F.get_or_null("sum", [], [col.Int64], False)])
    with pytest.raises(Unsupported):
        DistinctAggregator(bad)
    cnt = AggregatorParams([col.Int32], [F.get("count_distinct", [], [col.Int64]),
                                         F.get_or_null("count", [], [col.Int64], False)])
    DistinctAggregator(cnt)  # count never returns NULL: allowed
