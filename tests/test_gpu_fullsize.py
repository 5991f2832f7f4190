"""Every BASELINE.json config at the size bench.py measures it, checked on the device.

The oracle cannot hold 1e9-row inputs in seconds, so full-size results are checked against
reductions computed by torch directly over the input columns (sort / unique / bincount — none of
them goes through libdbgpu_agg), which pin the whole result, not just its totals:
  C2 (1e8 rows)  per-key counts from torch.bincount, and the oracle on all 1e8 rows;
  C3 (1e9 rows)  the full (UserID, count) set from torch.unique_consecutive over the sorted input;
  C4 (1e9 rows)  1e9 groups; rows sorted by WatchID give every group's ClientIP, COUNT = 1,
                 SUM(IsRefresh) and AVG(ResolutionWidth) exactly;
  C5 (1e9 rows)  per-phrase counts by the phrase's rank (bytes 0..4 are its base-26 digits,
                 include/dbgpu_datagen.h), every key's bytes against an input row of that phrase.
Each runs two steps through the bench's ConfigRunner (fresh table, then the reused/recycled one),
under AUTO (what bench.py runs) and, for the high-cardinality shapes, the radix-partitioned engine.
Oracle parity on the largest prefixes that finish in seconds is in test_prefix_vs_oracle.

Reference model for large known-answer checks: the 10M-row numbers() case of
tests/sqllogictests/suites/base/03_common/03_0043_new_agg_hashtable.test:116-124.
"""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd.filter import cmp
from oracle import oracle
from tests.parity import assert_results_equal
from tests.test_gpu_parity import oracle_aggregate

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _view(dcol, n, dtype):
    t = _torch()
    w = t.empty(0, dtype=dtype).element_size()
    return dcol.data[: n * w].view(dtype)


def _all_valid(dcol, n):
    t = _torch()
    if dcol.validity is None:
        return True
    full = n // 8
    ok = bool((dcol.validity[:full] == 255).all().item()) if full else True
    if n % 8:
        ok = ok and (int(dcol.validity[full].item()) & ((1 << (n % 8)) - 1)) == (1 << (n % 8)) - 1
    return ok


def _run(cfg, rows, strategy):
    from databend_amd import workloads
    r = workloads.ConfigRunner(cfg, rows, strategy=strategy)
    n0 = r.step(0)
    n1 = r.step(0)
    assert n0 == n1, f"second step over the same rows gave {n1} groups, first {n0}"
    return r, n1


def test_c2_full_100m():
    torch = _torch()
    from databend_amd import workloads
    rows = workloads.DEFAULT_ROWS[2]
    r, n = _run(2, rows, abi.STRATEGY_AUTO)
    try:
        adv = r.inputs[0]["AdvEngineID"].data.view(torch.int16)
        ref = torch.bincount(adv.to(torch.int64) + 32768, minlength=65536)
        ref[32768] = 0  # WHERE AdvEngineID <> 0
        keys = _view(r.out_keys[0], n, torch.int16).to(torch.int64) + 32768
        cnt = _view(r.out_aggs[0], n, torch.int64)
        got = torch.zeros(65536, dtype=torch.int64, device="cuda")
        got[keys] = cnt
        assert int((ref > 0).sum().item()) == n
        assert torch.equal(got, ref)
        assert int(cnt.sum().item()) == int((adv != 0).sum().item())
        # and the oracle over all 1e8 rows
        keys_h, aggs_h = r.results_host()
        cols = oracle.datagen(2, rows, threads=16)
        ok, oa = oracle_aggregate([cols["AdvEngineID"]], [("count", None)], (cmp(0, "<>", 0), [cols["AdvEngineID"]]),
                                  threads=16)
        assert_results_equal(keys_h, aggs_h, ok, oa)
    finally:
        r.close()


@pytest.mark.parametrize("strategy", [abi.STRATEGY_AUTO, abi.STRATEGY_PARTITIONED], ids=["auto", "partitioned"])
def test_c3_full_1b(strategy):
    torch = _torch()
    from databend_amd import workloads
    rows = workloads.DEFAULT_ROWS[3]
    r, n = _run(3, rows, strategy)
    try:
        uid = r.inputs[0]["UserID"].data.view(torch.int64)
        srt = torch.sort(uid).values
        ref_k, ref_c = torch.unique_consecutive(srt, return_counts=True)
        del srt
        assert n == ref_k.numel(), f"{n} groups, torch.unique says {ref_k.numel()}"
        keys = _view(r.out_keys[0], n, torch.int64)
        cnt = _view(r.out_aggs[0], n, torch.int64)
        ks, order = torch.sort(keys)
        assert torch.equal(ks, ref_k)
        assert torch.equal(cnt[order], ref_c)
        assert int(cnt.sum().item()) == rows
    finally:
        r.close()


@pytest.mark.parametrize("strategy", [abi.STRATEGY_AUTO], ids=["auto"])
def test_c4_full_1b(strategy):
    torch = _torch()
    from databend_amd import workloads
    rows = workloads.DEFAULT_ROWS[4]
    r, n = _run(4, rows, strategy)
    try:
        assert n == rows, f"WatchID is unique per row: expected {rows} groups, got {n}"
        inp = r.inputs[0]
        wid = inp["WatchID"].data.view(torch.int64)
        ws, wo = torch.sort(wid)
        assert bool((ws[1:] != ws[:-1]).all().item())
        del ws
        gw = _view(r.out_keys[0], n, torch.int64)
        gs, go = torch.sort(gw)
        del gs
        # every group, aligned by WatchID
        assert torch.equal(gw[go], wid[wo])
        assert torch.equal(_view(r.out_keys[1], n, torch.int32)[go], inp["ClientIP"].data.view(torch.int32)[wo])
        cnt = _view(r.out_aggs[0], n, torch.int64)
        assert bool((cnt == 1).all().item())
        s = _view(r.out_aggs[1], n, torch.int64)[go]
        assert torch.equal(s, inp["IsRefresh"].data.view(torch.int16)[wo].to(torch.int64))
        avg = _view(r.out_aggs[2], n, torch.float64)[go]
        assert torch.equal(avg, inp["ResolutionWidth"].data.view(torch.int16)[wo].to(torch.float64))
        for c in r.out_aggs:
            assert _all_valid(c, n)
        assert int(_view(r.out_aggs[1], n, torch.int64).sum().item()) == int(inp["IsRefresh"].data.view(torch.int16).to(torch.int64).sum().item())
    finally:
        r.close()


def _ranks(data, starts, torch):
    """Phrase rank from its first five bytes (base-26 digits of rank - 1, least significant first)."""
    r = torch.zeros(starts.numel(), dtype=torch.int64, device=starts.device)
    p = 1
    for j in range(5):
        r += (data[starts + j].to(torch.int64) - ord("a")) * p
        p *= 26
    return r + 1


@pytest.mark.parametrize("strategy", [abi.STRATEGY_AUTO, abi.STRATEGY_PARTITIONED], ids=["auto", "partitioned"])
def test_c5_full_1b(strategy):
    torch = _torch()
    from databend_amd import workloads
    rows = workloads.DEFAULT_ROWS[5]
    r, n = _run(5, rows, strategy)
    try:
        c = r.inputs[0]["SearchPhrase"]
        offs, data = c.offsets, c.data
        lens = offs[1:] - offs[:-1]
        sel = lens > 0
        n_sel = int(sel.sum().item())
        starts = offs[:-1][sel]
        ranks = _ranks(data, starts, torch)
        K = 1 << 23
        ref = torch.bincount(ranks, minlength=K + 1)
        rep = torch.empty(K + 1, dtype=torch.int64, device="cuda")
        rep[ranks] = starts  # one input row of each phrase
        rep_len = torch.zeros(K + 1, dtype=torch.int64, device="cuda")
        rep_len[ranks] = lens[sel]
        del ranks, sel
        assert n == int((ref > 0).sum().item())

        ko = r.out_keys[0].offsets[: n + 1]
        kd = r.out_keys[0].data
        klen = ko[1:] - ko[:-1]
        assert bool((klen > 0).all().item())
        gr = _ranks(kd, ko[:-1], torch)
        assert int(torch.bincount(gr, minlength=K + 1).max().item()) == 1, "a phrase appears in two groups"
        cnt = _view(r.out_aggs[0], n, torch.int64)
        got = torch.zeros(K + 1, dtype=torch.int64, device="cuda")
        got[gr] = cnt
        assert torch.equal(got, ref)
        assert int(cnt.sum().item()) == n_sel
        # key bytes: equal to an input occurrence of the same phrase
        assert torch.equal(klen, rep_len[gr])
        src = rep[gr]
        for j in range(32):
            m = klen > j
            if not bool(m.any().item()):
                break
            assert torch.equal(kd[ko[:-1][m] + j], data[src[m] + j]), f"key byte {j} differs"
    finally:
        r.close()


# Oracle parity on the largest prefixes that finish in seconds on the box's host cores.
@pytest.mark.parametrize("cfg,n", [(3, 100_000_000), (4, 40_000_000), (5, 200_000_000)])
def test_prefix_vs_oracle(cfg, n):
    from databend_amd import workloads
    res = workloads.run_config(cfg, n, steps=1)
    cols = oracle.datagen(cfg, n, threads=16)
    shape = workloads.SHAPES[cfg]
    filt = None
    if shape.predicate:
        name, op, const = shape.predicate
        filt = (cmp(0, op, const), [cols[name]])
    ok, oa = oracle_aggregate([cols[k] for k in shape.keys], [(f, cols[c] if c else None) for f, c in shape.aggs],
                              filt, threads=16)
    assert_results_equal(res["keys"], res["aggs"], ok, oa)
