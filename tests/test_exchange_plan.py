"""The before-partial shuffle's byte plan inside the library (dbg_payload_exchange_plan, the
function dbg_agg_exchange_payload follows) against databend_amd.exchange.payload_splits (the plan
the torch.distributed path and the gloo tests use), at world sizes 2..8, with the library's real
payload record widths for ClickBench Q33's shape (keys WatchID Int64 + ClientIP Int32; COUNT(*),
SUM(IsRefresh Int16), SQL AVG(ResolutionWidth Int16)).  Host only: no device work is called."""
import ctypes as C

import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregatorParams
from databend_amd.exchange import payload_owned, payload_splits
from databend_amd.ffi import check, lib

F = AggregateFunctionFactory.instance()


def _params():
    fns = [F.get("count"), F.get("sum", [], [col.Int16]), F.get("sql_avg", [], [col.Int16])]
    return AggregatorParams([col.Int64, col.Int32], fns)


@pytest.mark.parametrize("world", [2, 3, 4, 5, 7, 8])
def test_payload_plan_matches_python(world):
    rng = np.random.default_rng(world)
    all_counts = rng.integers(0, 1000, (world, 2, 256)).astype(np.uint64)
    all_counts[:, 1, rng.random(256) < 0.6] = 0
    p, keep = _params().to_abi(True, 0, -1)
    flat = np.ascontiguousarray(all_counts.reshape(-1))
    for rank in range(world):
        widths = (C.c_uint32 * 2)()
        send = (C.c_uint64 * (2 * world))()
        recv = (C.c_uint64 * (2 * world))()
        check(lib().dbg_payload_exchange_plan(C.byref(p), world, rank, flat.ctypes.data_as(C.POINTER(C.c_uint64)),
                                               widths, send, recv))
        w = (widths[0], widths[1])
        assert w[0] == 16 and w[1] % 8 == 0 and w[1] >= 16 + 8 * 4  # raw: 12-byte key + two Int16 args
        ps, pr = payload_splits(all_counts[rank], all_counts, w, rank, world)
        assert [list(send[k * world:(k + 1) * world]) for k in range(2)] == ps
        assert [list(recv[k * world:(k + 1) * world]) for k in range(2)] == pr
    # every byte sent is received exactly once, by the rank owning its partition
    for k in range(2):
        sent = sum(int(all_counts[r, k].sum()) for r in range(world))
        owned = sum(payload_owned(d, world)[1] - payload_owned(d, world)[0] for d in range(world))
        assert owned == 256 and sent == int(all_counts[:, k].sum())


def test_payload_plan_rejects_bad_arguments():
    from databend_amd.ffi import DbgError
    p, keep = _params().to_abi(True, 0, -1)
    counts = np.zeros(2 * 2 * 256, dtype=np.uint64)
    send = (C.c_uint64 * 4)()
    recv = (C.c_uint64 * 4)()
    with pytest.raises(DbgError):
        check(lib().dbg_payload_exchange_plan(C.byref(p), 2, 2, counts.ctypes.data_as(C.POINTER(C.c_uint64)), None, send, recv))


def _merge_params():
    """ClickBench Q13's partial shape (SearchPhrase String key; COUNT(*)) beside Q17's (UserID)."""
    return [AggregatorParams([col.String], [F.get("count")]),
            AggregatorParams([col.Int64], [F.get("count")]),
            AggregatorParams([col.Int64, col.Int32], [F.get("count"), F.get("sum", [], [col.Int16]), F.get("sql_avg", [], [col.Int16])])]


@pytest.mark.parametrize("world", [2, 3, 4, 5, 7, 8])
def test_merge_plan_matches_python(world):
    """The before_merge exchange's plan inside the library (dbg_merge_exchange_plan, the function
    dbg_agg_exchange follows) against databend_amd.exchange.merge_splits (the torch.distributed
    path's plan), with the library's record widths: every rank's send splits equal what each peer
    receives from it, in the peer's source order, and the sizes include self."""
    from databend_amd.exchange import merge_splits
    rng = np.random.default_rng(100 + world)
    for params in _merge_params():
        all_sizes = rng.integers(0, 5000, (world, world, 2)).astype(np.uint64)
        all_sizes[rng.random((world, world)) < 0.2] = 0  # empty segments, self included
        p, keep = params.to_abi(True, 0, -1)
        flat = np.ascontiguousarray(all_sizes.reshape(-1))
        plans = []
        for rank in range(world):
            w = C.c_uint32()
            send = (C.c_uint64 * (2 * world))()
            recv = (C.c_uint64 * (2 * world))()
            recs = (C.c_uint64 * world)()
            check(lib().dbg_merge_exchange_plan(C.byref(p), world, rank, flat.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                C.byref(w), send, recv, recs))
            width = w.value
            assert width % 8 == 0 and width >= 16
            counts, sbytes = all_sizes[rank, :, 0], all_sizes[rank, :, 1]
            got = [(int(all_sizes[s, rank, 0]), int(all_sizes[s, rank, 1])) for s in range(world)]
            sr, ss, rr, rs, seg = merge_splits(counts, sbytes, got, width)
            assert list(send[:world]) == sr and list(send[world:]) == ss
            assert list(recv[:world]) == rr and list(recv[world:]) == rs and list(recs) == seg
            plans.append((list(send), list(recv)))
        for a in range(world):  # a's send to b is b's receive from a
            for b in range(world):
                assert plans[a][0][b] == plans[b][1][a] and plans[a][0][world + b] == plans[b][1][world + a]


def test_merge_plan_rejects_bad_arguments():
    from databend_amd.ffi import DbgError
    p, keep = _merge_params()[1].to_abi(True, 0, -1)
    sizes = np.zeros(2 * 2 * 2, dtype=np.uint64)
    send, recv, recs = (C.c_uint64 * 4)(), (C.c_uint64 * 4)(), (C.c_uint64 * 2)()
    with pytest.raises(DbgError):
        check(lib().dbg_merge_exchange_plan(C.byref(p), 2, 2, sizes.ctypes.data_as(C.POINTER(C.c_uint64)), None, send, recv, recs))
