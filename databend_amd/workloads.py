"""The five benchmark configurations of BASELINE.json / SURVEY.md §8d on the GPU path.

Each config = input columns (generated in HBM by `dbg_datagen`, the numbers_mt analog), group
columns, aggregate functions and an optional WHERE predicate — the query shapes of
ClickBench 07.sql / 12.sql / 15.sql / 32.sql and TPC-H Q1 (benchmark/clickbench/hits/queries,
tests/sqllogictests/suites/tpch/queries.test:31-58).

`run_config` is one "step" of the hot path per batch: fresh table -> fused filter + GROUP BY over
all rows -> result columns resident in HBM.  Used by bench.py and the GPU tests.
"""
from __future__ import annotations

import ctypes as C
import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from . import abi
from . import column as col
from .aggregates import AggregateFunctionFactory
from .aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from .column import Column, DataType
from .device import DeviceColumn, empty
from .ffi import check, lib
from .filter import FilterProgram, cmp

BASE_SEED = 0xDA7ABE7D
F = AggregateFunctionFactory.instance()


def _torch():
    import torch
    return torch


_C5_CDF = None


def c5_cdf_device():
    """The exact integer Zipf CDF of include/dbgpu_datagen.h, built on the host (numpy) and
    uploaded once (64 MiB)."""
    global _C5_CDF
    if _C5_CDF is None:
        torch = _torch()
        r = np.arange(1, (1 << 23) + 1, dtype=np.uint64)
        w = (np.uint64(1) << np.uint64(40)) // r
        cdf = np.cumsum(w, dtype=np.uint64)
        _C5_CDF = torch.from_numpy(cdf.view(np.int64)).cuda()
    return _C5_CDF


def _gen(cfg: int, seed: int, start: int, rows: int, outs, aux=None):
    torch = _torch()
    arr = (C.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
    check(lib().dbg_datagen(cfg, seed, start, rows, arr, len(outs), aux.data_ptr() if aux is not None else None,
                            torch.cuda.current_stream().cuda_stream))


def generate_device(cfg: int, rows: int, start: int = 0, seed: Optional[int] = None) -> Dict[str, DeviceColumn]:
    """Device columns of config cfg for rows [start, start+rows) — equal to oracle.datagen."""
    torch = _torch()
    seed = BASE_SEED + cfg if seed is None else seed
    dev = "cuda"
    u8 = lambda n: torch.empty(max(1, n), dtype=torch.uint8, device=dev)
    if cfg == 1:
        ship = u8(rows * 4)
        rf, ls = u8(rows), u8(rows)
        rfo = torch.empty(rows + 1, dtype=torch.int64, device=dev)
        lso = torch.empty(rows + 1, dtype=torch.int64, device=dev)
        decs = [u8(rows * 16) for _ in range(6)]
        _gen(1, seed, start, rows, [ship, rf, ls, rfo, lso] + decs)
        d = lambda t, p, s: DeviceColumn(col.Decimal128(p, s), t, None, None, rows)
        return {
            "l_shipdate": DeviceColumn(col.Date, ship, None, None, rows),
            "l_returnflag": DeviceColumn(col.String, rf, rfo, None, rows),
            "l_linestatus": DeviceColumn(col.String, ls, lso, None, rows),
            "l_quantity": d(decs[0], 15, 2), "l_extendedprice": d(decs[1], 15, 2),
            "l_discount": d(decs[2], 15, 2), "l_tax": d(decs[3], 15, 2),
            "disc_price": d(decs[4], 31, 4), "charge": d(decs[5], 38, 6),
        }
    if cfg == 2:
        b = u8(rows * 2)
        _gen(2, seed, start, rows, [b])
        return {"AdvEngineID": DeviceColumn(col.Int16, b, None, None, rows)}
    if cfg == 3:
        b = u8(rows * 8)
        _gen(3, seed, start, rows, [b])
        return {"UserID": DeviceColumn(col.Int64, b, None, None, rows)}
    if cfg == 4:
        bs = [u8(rows * 8), u8(rows * 4), u8(rows * 2), u8(rows * 2)]
        _gen(4, seed, start, rows, bs)
        return {"WatchID": DeviceColumn(col.Int64, bs[0], None, None, rows),
                "ClientIP": DeviceColumn(col.Int32, bs[1], None, None, rows),
                "IsRefresh": DeviceColumn(col.Int16, bs[2], None, None, rows),
                "ResolutionWidth": DeviceColumn(col.Int16, bs[3], None, None, rows)}
    if cfg == 5:
        cdf = c5_cdf_device()
        lens = torch.empty(rows, dtype=torch.int64, device=dev)
        _gen(5, seed, start, rows, [lens], cdf)
        offs = torch.zeros(rows + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=offs[1:])
        total = int(offs[-1].item())
        data = u8(total)
        _gen(6, seed, start, rows, [offs, data], cdf)
        del lens
        return {"SearchPhrase": DeviceColumn(col.String, data, offs, None, rows)}
    raise ValueError(cfg)


@dataclass
class QueryShape:
    name: str
    keys: List[str]
    aggs: List[tuple]          # (function name, column name or None)
    predicate: Optional[tuple]  # (column name, op, constant)
    sql: str


SHAPES = {
    1: QueryShape("tpch_q1_sf1", ["l_returnflag", "l_linestatus"],
                  [("sum", "l_quantity"), ("sum", "l_extendedprice"), ("sum", "disc_price"), ("sum", "charge"),
                   ("sql_avg", "l_quantity"), ("sql_avg", "l_extendedprice"), ("sql_avg", "l_discount"), ("count", None)],
                  ("l_shipdate", "<=", 10471),
                  "TPC-H Q1: WHERE l_shipdate <= DATE '1998-09-02' GROUP BY l_returnflag, l_linestatus"),
    2: QueryShape("clickbench_q8_adv_engine_id", ["AdvEngineID"], [("count", None)], ("AdvEngineID", "<>", 0),
                  "SELECT AdvEngineID, COUNT(*) FROM hits WHERE AdvEngineID <> 0 GROUP BY AdvEngineID"),
    3: QueryShape("clickbench_q17_user_id", ["UserID"], [("count", None)], None,
                  "SELECT UserID, COUNT(*) FROM hits GROUP BY UserID"),
    4: QueryShape("clickbench_q33_watchid_clientip", ["WatchID", "ClientIP"],
                  [("count", None), ("sum", "IsRefresh"), ("sql_avg", "ResolutionWidth")], None,
                  "SELECT WatchID, ClientIP, COUNT(*), SUM(IsRefresh), AVG(ResolutionWidth) FROM hits GROUP BY WatchID, ClientIP"),
    5: QueryShape("clickbench_q13_search_phrase", ["SearchPhrase"], [("count", None)], ("SearchPhrase", "<>", ""),
                  "SELECT SearchPhrase, COUNT(*) FROM hits WHERE SearchPhrase <> '' GROUP BY SearchPhrase"),
}
DEFAULT_ROWS = {1: 6_001_215, 2: 100_000_000, 3: 1_000_000_000, 4: 1_000_000_000, 5: 1_000_000_000}


def params_for(cfg: int, types: Dict[str, DataType]) -> AggregatorParams:
    shape = SHAPES[cfg]
    fns = [F.get(f, [], [types[c]] if c else []) for f, c in shape.aggs]
    return AggregatorParams([types[k] for k in shape.keys], fns)


def col_bytes(c, rows_counted: int) -> int:
    """Bytes of a column for `rows_counted` rows (strings: 8-byte offset + mean payload)."""
    if c.dtype.type_id == abi.STRING:
        total = int(c.offsets[-1].item()) if hasattr(c.offsets, "item") else int(c.offsets[-1])
        return rows_counted * 8 + int(round(total * rows_counted / max(1, len(c))))
    return rows_counted * c.dtype.width


def algorithmic_bytes(cfg: int, cols: Dict[str, DeviceColumn], n_rows: int, n_selected: int, n_groups: int,
                      result_types: List[DataType], key_string_bytes: int) -> int:
    """predicate columns over all N rows + key/argument columns over the selected
    rows (each distinct column once) + G x (key widths + result widths)."""
    shape = SHAPES[cfg]
    b = 0
    seen = set()
    if shape.predicate:
        pc = shape.predicate[0]
        b += col_bytes(cols[pc], n_rows)
        seen.add(pc)
    for name in list(shape.keys) + [c for _, c in shape.aggs if c]:
        if name in seen:
            continue
        seen.add(name)
        b += col_bytes(cols[name], n_selected)
    for k in shape.keys:
        t = cols[k].dtype
        b += n_groups * (8 if t.type_id == abi.STRING else t.width)
    b += key_string_bytes
    for t in result_types:
        b += n_groups * t.width
    return b


class ConfigRunner:
    """Holds device inputs (several rotating copies so the timed loop is not served from the
    256 MiB Infinity Cache) and one reusable GPU table for config cfg."""

    def __init__(self, cfg: int, rows: int, copies: int = 1, capacity_hint: int = 0, seed: Optional[int] = None,
                 start: int = 0, strategy: int = abi.STRATEGY_AUTO):
        torch = _torch()
        self.cfg, self.rows = cfg, rows
        self.shape = SHAPES[cfg]
        self.inputs = [generate_device(cfg, rows, start=start + k * rows, seed=seed) for k in range(copies)]
        torch.cuda.synchronize()
        types = {k: v.dtype for k, v in self.inputs[0].items()}
        self.params = params_for(cfg, types)
        self.result_types = [f.return_type() for f in self.params.aggregate_functions]
        self._capacity_hint = capacity_hint
        self.table = AggregateHashTable(self.params, HashTableConfig(True, capacity_hint))
        self.table.set_strategy(strategy)
        # one table per batch stream: a small table is re-initialised by the fused finalize
        check(lib().dbg_agg_set_recycle(self.table.h, 1))
        self.programs = []
        for inp in self.inputs:
            if self.shape.predicate:
                name, op, const = self.shape.predicate
                self.programs.append(FilterProgram(cmp(0, op, const), [inp[name]]))
            else:
                self.programs.append(None)
        self.key_abi = [[inp[k] for k in self.shape.keys] for inp in self.inputs]
        self.arg_cols = [[None if c is None else inp[c] for _, c in self.shape.aggs] for inp in self.inputs]
        self.out = None

    def _prepared(self, i):
        """The C-ABI argument structs of input copy i, built once (host-side marshalling is not
        part of the hot path)."""
        cache = getattr(self, "_prep", None)
        if cache is None:
            cache = self._prep = {}
        if i not in cache:
            from .column import abi_array
            keys = abi_array([c.to_abi() for c in self.key_abi[i]])
            args = []
            for c in self.arg_cols[i]:
                if c is None:
                    d = abi.dbg_column()
                    d.dt = abi.dbg_datatype(-1, 0, 0, 0, 0)
                    args.append(d)
                else:
                    args.append(c.to_abi())
            args = abi_array(args)
            fp = self.programs[i].ptr() if self.programs[i] is not None else None
            cache[i] = (keys, args, fp)
        return cache[i]

    def step(self, k: int = 0):
        """One pass of the hot path over one batch; results land in HBM (self.out_*).
        reset -> fused filter + GROUP BY insert -> fused finalize (count, scan, write) with one
        host round trip (dbg_agg_finalize_into)."""
        self.insert(k)
        return self.finalize_into(self.table.h)

    def insert(self, k: int = 0, table=None):
        """reset -> fused filter + GROUP BY insert of input copy k into the partial table."""
        i = k % len(self.inputs)
        L = lib()
        h = (table or self.table).h
        keys, args, fp = self._prepared(i)
        check(L.dbg_agg_reset(h))
        check(L.dbg_agg_add_groups(h, keys, args, fp, self.rows, 1))

    # ---- output columns (one set per pipeline parity)
    def _outset(self, parity=0):
        sets = self.__dict__.setdefault("_outsets", {})
        if parity not in sets:
            sets[parity] = _OutSet(self, 4096, [1 << 16] * len(self.shape.keys))
        return sets[parity]

    def _alloc_out(self, cap, scap, parity=0):
        self.__dict__.setdefault("_outsets", {})[parity] = _OutSet(self, cap, scap)

    def _publish(self, o, n, sb):
        self.n_groups, self.key_string_bytes = n, sum(sb)
        self.out_aggs, self.out_keys = o.aggs, o.keys
        for c in o.aggs + o.keys:
            c.length = n
        return n

    def finalize_into(self, h, parity=0):
        """Fused finalize of table handle h into this runner's device output columns."""
        L = lib()
        n = C.c_uint64()
        sb = (C.c_uint64 * len(self.shape.keys))()
        for _ in range(2):
            o = self._outset(parity)
            rc = L.dbg_agg_finalize_into(h, o.oa, o.ok, o.cap, o.scap, C.byref(n), sb)
            if rc == abi.DBG_ERR_INVALID and (n.value > o.cap or any(x > y for x, y in zip(sb, o.scap))):
                self._alloc_out(int(n.value * 1.25) + 1, [int(x * 1.25) + 1 for x in sb], parity)
                continue
            check(rc)
            break
        return self._publish(o, n.value, list(sb))

    def finalize_async(self, h, parity=0):
        o = self._outset(parity)
        check(lib().dbg_agg_finalize_into_async(h, o.oa, o.ok, o.cap, o.scap))

    def finalize_wait(self, h, parity=0):
        n = C.c_uint64()
        sb = (C.c_uint64 * len(self.shape.keys))()
        o = self._outset(parity)
        rc = lib().dbg_agg_finalize_wait(h, C.byref(n), sb)
        if rc == abi.DBG_ERR_INVALID and (n.value > o.cap or any(x > y for x, y in zip(sb, o.scap))):
            # buffers too short: the table is intact (no recycle), finalize again into larger ones
            self._alloc_out(int(n.value * 1.25) + 1, [int(x * 1.25) + 1 for x in sb], parity)
            return self.finalize_into(h, parity)
        check(rc)
        return self._publish(o, n.value, list(sb))

    # ---- pipelined steps: batch k's finalize overlaps batch k+1's insert
    def enable_pipeline(self, mode: str = ""):
        """Two partial tables used alternately, the host enqueueing batch k+1 before it waits for
        batch k's finalize, so the GPU never idles on the host between batches.
          single : both tables on one stream — the batches run strictly in sequence (default)
          dual   : table k % 2 on stream k % 2 (no cross-stream events: each table's insert and
                   finalize stay on its own stream); consecutive batches may overlap
        Cross-stream event hand-offs cost ~10 us each on this platform (measured), more than the
        13 us finalize they would hide, so no mode uses them."""
        import os
        torch = _torch()
        if getattr(self, "tables", None):
            return
        self.pipe_mode = mode or os.environ.get("DBG_PIPE_MODE", "single")
        t1 = AggregateHashTable(self.params, HashTableConfig(True, self._capacity_hint))
        check(lib().dbg_agg_set_recycle(t1.h, 1))
        self.tables = [self.table, t1]
        sa = torch.cuda.Stream()
        self.streams = [sa, sa if self.pipe_mode == "single" else torch.cuda.Stream()]
        for t, st in zip(self.tables, self.streams):
            t.set_stream(st)
        self._inflight = None

    def pipe_step(self, k: int):
        p = k % 2
        t = self.tables[p]
        self.insert(k, t)
        self.finalize_async(t.h, p)
        n = self.pipe_drain()
        self._inflight = (t.h, p)
        return n

    def pipe_drain(self):
        """Complete the finalize in flight (if any); returns its group count."""
        f, self._inflight = getattr(self, "_inflight", None), None
        return self.finalize_wait(*f) if f else 0

    def results_host(self):
        keys = [c.to_host_n(self.n_groups) if hasattr(c, "to_host_n") else _dev_to_host(c, self.n_groups) for c in self.out_keys]
        aggs = [_dev_to_host(c, self.n_groups) for c in self.out_aggs]
        return keys, aggs

    def close(self):
        for t in getattr(self, "tables", None) or [self.table]:
            t.close()


class _OutSet:
    """Device output columns + their C-ABI structs for one fused finalize."""

    def __init__(self, runner, cap, scap):
        self.aggs = [empty(t, cap) for t in runner.result_types]
        self.keys = [empty(t, cap, string_bytes=scap[j]) for j, t in enumerate(runner.params.group_data_types)]
        self.oa = (abi.dbg_out_column * len(self.aggs))()
        self.ok = (abi.dbg_out_column * len(self.keys))()
        for j, c in enumerate(self.aggs):
            self.oa[j].data = c.data.data_ptr()
            self.oa[j].validity = c.validity.data_ptr() if c.validity is not None else None
        for j, c in enumerate(self.keys):
            self.ok[j].data = c.data.data_ptr()
            self.ok[j].offsets = c.offsets.data_ptr() if c.offsets is not None else None
            self.ok[j].validity = c.validity.data_ptr() if c.validity is not None else None
        self.cap = cap
        self.scap = (C.c_uint64 * len(scap))(*scap)


def _dev_to_host(c: DeviceColumn, n: int) -> Column:
    t = c.dtype
    if t.type_id == abi.STRING:
        offs = c.offsets[: n + 1].cpu().numpy().view(np.uint64).copy()
        data = c.data[: int(offs[-1]) if n else 0].cpu().numpy().copy()
    else:
        offs = None
        data = c.data[: n * t.width].cpu().numpy().copy()
        if t.type_id not in (abi.DECIMAL128,):
            data = data.view(t.np_dtype)
    val = None
    if t.nullable and c.validity is not None:
        val = np.unpackbits(c.validity.cpu().numpy(), bitorder="little")[:n].astype(bool)
    return Column(t, data, offs, val)


def run_config(cfg: int, rows: int, steps: int = 1, copies: int = 1, capacity_hint: int = 0,
               strategy: int = abi.STRATEGY_AUTO) -> dict:
    torch = _torch()
    r = ConfigRunner(cfg, rows, copies=copies, capacity_hint=capacity_hint, strategy=strategy)
    try:
        times = []
        for k in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.step(k)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        keys, aggs = r.results_host()
        part, rounds = r.table.strategy()
        return dict(keys=keys, aggs=aggs, n_groups=r.n_groups, times=times, partitioned=part, extra_rounds=rounds)
    finally:
        r.close()
