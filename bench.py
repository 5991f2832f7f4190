"""bench.py — the reference's headline metric on MI355X: input rows/s aggregated + % of HBM roofline.

Default workload (BASELINE.json configs[1]): ClickBench Q8-style
    SELECT AdvEngineID, COUNT(*) FROM hits WHERE AdvEngineID <> 0 GROUP BY AdvEngineID
over 100M synthetic rows per GPU (AdvEngineID Int16, P(0) = 0.9937).  One step = one pass of the
hot path over one batch: fresh table -> fused filter + GROUP BY over every row -> (N > 1: partial
states gathered (low cardinality) or routed by hash % N (high) over RCCL and merged) -> result
columns resident in HBM.  Consecutive batches are pipelined on two streams (batch k's finalize /
exchange overlaps batch k+1's insert; two tables alternate); every batch's work completes inside
the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1..5] [--rows R]

Multi-GPU: launched by torch.distributed.run, one rank per GPU (backend nccl = RCCL); every rank
aggregates its own 100M rows (weak scaling), timing = max over ranks, value = all ranks' rows / time.
Rank 0 prints ONE JSON line.  See DESIGN.md for the roofline accounting.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", type=int, default=2)
    p.add_argument("--rows", type=int, default=0, help="rows per GPU (default: the config's size)")
    p.add_argument("--copies", type=int, default=0, help="rotating input copies (default: enough to defeat the 256 MiB L3)")
    p.add_argument("--cpu-sample-rows", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--capacity-hint", type=int, default=0)
    p.add_argument("--strategy", choices=["auto", "table", "partitioned"], default="auto",
                   help="aggregation strategy of the tables (dbg_agg_set_strategy); auto = the cardinality probe")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher plumbing only: every rank joins a gloo group, rank 0 prints n_gpus (no GPU work)")
    p.add_argument("--extra-configs", default=None,
                   help="comma list of further configs timed in the same run (single GPU), reported under 'configs' "
                        "(default: 1,3,4,5 with the headline config 2 at N=1; none otherwise; 'none' disables)")
    p.add_argument("--extra-steps", type=int, default=3)
    p.add_argument("--exchange", choices=["abi", "torch"], default="abi",
                   help="N > 1, high cardinality: the library's RCCL exchange (dbg_agg_exchange / "
                        "dbg_agg_exchange_payload, what a Rust host drives) or torch.distributed all-to-all")
    p.add_argument("--shuffle-chunks", type=int, default=4,
                   help="before_partial at N > 1: add_groups in this many row chunks, each chunk's level-1 "
                        "records shipped while the next chunk is scattered (dbg_agg_exchange_payload_chunk)")
    p.add_argument("--shuffle", choices=["auto", "before_partial", "before_merge"], default="auto",
                   help="N > 1, high cardinality: route level-1 records before any aggregation (group_by_shuffle_mode "
                        "= before_partial, partitioned payload) or partial states after it; auto = before_partial when, "
                        "on every rank, the probe chose the partitioned payload or the rows' raw records are fewer "
                        "bytes than the rank's group records (exchange.prefer_before_partial)")
    p.add_argument("--scaling", choices=["weak", "strong"], default=None,
                   help="weak: every GPU aggregates the config's rows; strong: the config's rows are split over "
                        "the GPUs (default: strong for the 1B-row configs 3-5, weak for 1-2)")
    return p.parse_args()


def cpu_baseline(cfg, sample_rows, gpu_check=None):
    """Restated Databend CPU aggregator (oracle/, the reference's algorithm: per-thread partial
    AggregateHashTable over 65536-row blocks -> partition bucket -> final) on the host's cores,
    on a bounded sample of the same workload; median of 5 timed runs after 1 warm-up."""
    from oracle import oracle
    from databend_amd.workloads import SHAPES, F
    from databend_amd.filter import FilterProgram, cmp
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))  # the GPU box grants 16 CPUs per GPU
    shape = SHAPES[cfg]
    cols = oracle.datagen(cfg, sample_rows, threads=threads)
    keys = [cols[k] for k in shape.keys]
    aggs = [(F.get(f, [], [cols[c].dtype] if c else []).to_abi(), cols[c] if c else None) for f, c in shape.aggs]
    prog = None
    if shape.predicate:
        name, op, const = shape.predicate
        prog = FilterProgram(cmp(0, op, const), [cols[name].to_abi()])
    times = []
    result = None
    for it in range(6):
        t0 = time.perf_counter()
        result = oracle.aggregate(keys, aggs, filter_program=prog, threads=threads)
        dt = time.perf_counter() - t0
        if it:
            times.append(dt)
    med = statistics.median(times)
    n_groups = len(result[0][0]) if result and result[0] else 0
    return dict(value=sample_rows / med, unit="rows/s", cores=threads, kind="port",
                label="restated Databend CPU aggregator (oracle/dbagg_oracle.cpp: per-thread partial "
                      "AggregateHashTable -> partition bucket -> final)",
                sample=f"{sample_rows} rows of the same synthetic workload (rows 0..{sample_rows - 1}, "
                       f"{n_groups} groups), median of {len(times)} runs after 1 warm-up, {threads} threads",
                sample_groups=n_groups, seconds_per_run=med), result, cols


def spawn_ranks(args) -> int:
    """`--gpus N` without a launcher: start `torch.distributed.run` with N ranks (one per GPU) as a
    child process before this process touches the GPU (never exec), relay its output (rank 0 prints
    the JSON line) and return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def load_traffic(cfg):
    """PMC-measured HBM bytes per step / launch (scripts/pmc_step_traffic.py, profiles/)."""
    tf = os.path.join(ROOT, "profiles", f"pmc_traffic_c{cfg}.json")
    if not os.path.exists(tf):
        return None, None
    try:
        t = json.load(open(tf))
        return t.get("hbm_bytes_per_launch"), os.path.relpath(tf, ROOT)
    except Exception:
        return None, None


def measure_extra(cfg, steps, warmup, with_cpu):
    """One more configuration at its full size on this GPU (single rank): the same step as the
    headline (reset -> fused filter + GROUP BY -> finalize into HBM result columns), timed over
    `steps` steps after `warmup`, its roofline over the whole step's kernels (from
    the first launch to result columns in HBM), and the CPU baseline on a bounded sample."""
    import torch
    from databend_amd import ffi
    from databend_amd.workloads import DEFAULT_ROWS, SHAPES, ConfigRunner, algorithmic_bytes
    rows = DEFAULT_ROWS[cfg]
    shape = SHAPES[cfg]
    copies = 2 if cfg == 1 else 1  # C1's 600 MB would sit in the 256 MiB L3 less than twice over
    runner = ConfigRunner(cfg, rows, copies=copies)
    try:
        for k in range(warmup):
            runner.step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            runner.step(warmup + k)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ffi.prof_reset()
        ffi.prof_enable(True)
        for k in range(steps):
            runner.step(warmup + steps + k)
        torch.cuda.synchronize()
        ffi.prof_enable(False)
        prof = ffi.prof_read()
        step_kernel_ms = sum(v[0] for v in prof.values()) / steps
        n_groups = runner.n_groups
        ci = next((i for i, (f, c) in enumerate(shape.aggs) if f == "count" and c is None), None)
        sel = int(runner.out_aggs[ci].data[: 8 * n_groups].view(torch.int64).sum().item()) if ci is not None else rows
        alg = algorithmic_bytes(cfg, runner.inputs[0], rows, sel, n_groups, runner.result_types, runner.key_string_bytes)
        achieved = alg / (step_kernel_ms * 1e-3) / 1e9 if step_kernel_ms > 0 else 0.0
        traffic, tsrc = load_traffic(cfg)
        partitioned = runner.table.strategy()[0]
        dom = max(prof.items(), key=lambda kv: kv[1][0])[0] if prof else None
        rec = {
            "workload": shape.name, "query": shape.sql, "rows": rows, "groups": n_groups, "selected_rows": sel,
            "strategy": "partitioned" if partitioned else "hbm_table",
            "steps": steps, "warmup": warmup, "ms_per_step": elapsed / steps * 1e3, "rows_per_s": rows * steps / elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                         "kernel": "step (every kernel of one step)", "kernel_avg_ms": step_kernel_ms,
                         "algorithmic_bytes_per_launch": alg,
                         "traffic_over_algorithmic": traffic / alg if traffic else None},
            "dominant_kernel": dom,
            "kernels_ms_per_step": {k: v[0] / steps for k, v in prof.items()},
        }
    finally:
        runner.close()
        del runner
        torch.cuda.empty_cache()
    if with_cpu:
        sample = {1: 6_001_215, 3: 20_000_000, 4: 10_000_000, 5: 20_000_000}[cfg]
        cb, _, _ = cpu_baseline(cfg, sample)
        rec["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "label", "sample", "sample_groups")}
        # the GPU's groups beside the sample's: a sample holds fewer groups than the full config
        rec["cpu_baseline"]["full_config_groups"] = n_groups
        rec["gpu_vs_cpu"] = rec["rows_per_s"] / cb["value"]
    return rec


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    if args.dry_run:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        if world > 1:
            dist.init_process_group("gloo")
            seen = torch.tensor([1])
            dist.all_reduce(seen)
            world_seen = int(seen.item())
            dist.destroy_process_group()
        else:
            world_seen = 1
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world_seen, "gpus_requested": args.gpus}), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=dev)

    from databend_amd import ffi
    from databend_amd.aggregator import AggregateHashTable, HashTableConfig
    from databend_amd import abi
    from databend_amd.exchange import AbiComm, GatherPipeline, exchange_partial, exchange_payload
    from databend_amd.workloads import DEFAULT_ROWS, SHAPES, ConfigRunner, algorithmic_bytes

    cfg = args.config
    scaling = args.scaling or ("strong" if cfg in (3, 4, 5) else "weak")
    total_rows = args.rows or DEFAULT_ROWS[cfg]
    # strong scaling: the config's rows split over the ranks; weak: every rank its own full batch
    rows = total_rows // world if scaling == "strong" else total_rows
    shape = SHAPES[cfg]
    in_bytes_per_row = {1: 100, 2: 2, 3: 8, 4: 16, 5: 27}[cfg]
    copies = args.copies or max(1, min(4, -(-768 * 2**20 // max(1, rows * in_bytes_per_row))))
    if cfg in (3, 4, 5):
        copies = args.copies or 1
    # rank r aggregates its own disjoint rows of the synthetic table (weak scaling)
    # every rank aggregates disjoint row ranges of the same generator
    strategy = {"auto": abi.STRATEGY_AUTO, "table": abi.STRATEGY_TABLE, "partitioned": abi.STRATEGY_PARTITIONED}[args.strategy]
    runner = ConfigRunner(cfg, rows, copies=copies, capacity_hint=args.capacity_hint, start=rank * copies * rows,
                          strategy=strategy)
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)", file=sys.stderr)
    final = None
    small = False
    if world > 1:
        final = AggregateHashTable(runner.params, HashTableConfig(False, args.capacity_hint))
        final.set_strategy(strategy)
        ffi.check(ffi.lib().dbg_agg_set_recycle(final.h, 1))
        # low cardinality: replicas + gather to rank 0 over one RCCL all-gather;
        # otherwise partial states routed by hash % N with all-to-all (exchange_partial)
        small = bool(shape.keys) and all(runner.inputs[0][k].dtype.width in (1, 2, 4, 8) and
                                         runner.inputs[0][k].dtype.type_id != abi.STRING for k in shape.keys) \
            and len(shape.keys) == 1 and runner.table.capacity <= 8192

    # Batches are pipelined: batch k's finalize (and, N > 1, its exchange and
    # final merge) overlaps batch k+1's insert on a second stream; drain() completes the last
    # one inside the timed region.
    # Pipelining pays where a step is tens of microseconds (C1, C2).  A high-cardinality step is
    # milliseconds of GPU work per launch, and a second table of its size (C4: 2^31 slots x 64 B)
    # would not fit next to the first, so those run one table, step after step.
    pipe = None
    pipelined = world == 1 and cfg in (1, 2)
    if pipelined:
        runner.enable_pipeline()
    elif small:
        pipe = GatherPipeline(runner, final, dev, rank, world)

    # High cardinality at N > 1: decide the shuffle once, the same on every rank (one untimed
    # insert shows what each rank's cardinality probe chose), then keep the table in that mode.
    comm = None
    before_partial = False
    if world > 1 and not small:
        if args.exchange == "abi":
            comm = AbiComm.from_process_group(local)
        t = runner.table
        t.reset()
        t.add_groups(runner.key_abi[0], runner.arg_cols[0], rows=rows, filter_program=runner.programs[0], on_device=True)
        fixed = all(runner.inputs[0][k].dtype.type_id != abi.STRING for k in shape.keys)
        # before_partial when shipping the rows is fewer bytes than shipping this rank's groups
        # (exchange.prefer_before_partial), or when the probe already chose the partitioned payload;
        # the same choice on every rank (one all-reduce, untimed).  String keys stay before_merge
        # (a payload record references a local row).
        from databend_amd.exchange import payload_widths, prefer_before_partial
        want = bool(t.strategy()[0])
        if fixed and not want:
            want = prefer_before_partial(rows, t.finalize()[0], payload_widths(runner.params))
        vote = torch.tensor([1 if (want and fixed) else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(vote, op=dist.ReduceOp.MIN)
        before_partial = args.shuffle == "before_partial" or (args.shuffle == "auto" and int(vote.item()) == 1)
        t.reset()
        if before_partial:
            t.set_strategy(abi.STRATEGY_PARTITIONED)

    def drain():
        if pipelined:
            return runner.pipe_drain()
        if pipe is not None:
            return pipe.drain()
        return 0

    def dslice(c, lo, hi):  # rows [lo, hi) of a fixed-width non-null device column (a view)
        from databend_amd.device import DeviceColumn
        w = c.dtype.width
        return DeviceColumn(c.dtype, c.data[lo * w:hi * w], None, None, hi - lo)

    def chunked_shuffle(t, i):
        """add_groups in row chunks, each chunk's level-1 records shipped while the next scatters."""
        from databend_amd.exchange import PayloadShuffle
        nchunk = args.shuffle_chunks
        sh = None if comm is not None else PayloadShuffle(t, dev)
        for c in range(nchunk):
            lo, hi = (rows * c // nchunk) & ~7, (rows if c + 1 == nchunk else (rows * (c + 1) // nchunk) & ~7)
            t.add_groups([dslice(x, lo, hi) for x in runner.key_abi[i]],
                         [None if x is None else dslice(x, lo, hi) for x in runner.arg_cols[i]], rows=hi - lo, on_device=True)
            if comm is not None:
                comm.exchange_payload_chunk(t, last=c + 1 == nchunk)
            else:
                sh.ship()
        if sh is not None:
            sh.finish()

    def chunkable(i):
        cols = list(runner.key_abi[i]) + [x for x in runner.arg_cols[i] if x is not None]
        return args.shuffle_chunks > 1 and runner.programs[i] is None and all(
            x.dtype.width in (1, 2, 4, 8) and not x.dtype.nullable and x.offsets is None for x in cols)

    def step(k):
        if pipelined:
            return runner.pipe_step(k)
        if world == 1:
            return runner.step(k)
        if pipe is not None:
            return pipe.step(k)
        i = k % len(runner.inputs)
        t = runner.table
        t.reset()
        if before_partial and chunkable(i):  # the shuffle overlapped with level 1, chunk by chunk
            chunked_shuffle(t, i)
            n, sb = t.finalize()
            return n
        t.add_groups(runner.key_abi[i], runner.arg_cols[i], rows=rows, filter_program=runner.programs[i], on_device=True)
        if before_partial:  # level-1 records to their partition's owner, aggregated once there
            if comm is not None:
                comm.exchange_payload(t)
            else:
                exchange_payload(t, dev)
            n, sb = t.finalize()
            return n
        final.reset()
        if comm is not None:
            comm.exchange(t, final)
        else:
            exchange_partial(t, final, dev)
        n, sb = final.finalize()
        return n

    for k in range(args.warmup):
        step(k)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    drain()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    # Kernel durations for the roofline: a second pass of the same steps with HIP events recorded
    # around every launch on the stream it runs on (dbg_prof_enable).  Kept out of the timed pass
    # above: event records add host and GPU work between launches.
    ffi.prof_reset()
    ffi.prof_enable(True)
    for k in range(args.steps):
        step(args.warmup + args.steps + k)
    drain()
    torch.cuda.synchronize()
    ffi.prof_enable(False)
    prof = ffi.prof_read()

    # dominant kernel: the fused filter + GROUP BY insert (HBM-table strategy), or — radix-
    # partitioned strategy (pp.hip, high cardinality) — the whole step's level passes + LDS
    # aggregation, whose launches together touch the §8d bytes once
    partitioned = runner.table.strategy()[0]
    if partitioned:
        pp_names = [k for k in prof if k.startswith("pp_") and k != "pp_probe"]
        ins_ms = sum(prof[k][0] for k in pp_names)
        ins_n = args.steps
        kernel_name = "+".join(sorted(pp_names)) + " (one step)"
    else:
        ins_ms, ins_n = prof.get("agg_insert", (0.0, 0))
        kernel_name = "agg_insert"
        if "part_direct" in prof:  # C3: the sort in the insert, the table stage in the finalize (part.hip)
            ins_ms += prof["part_direct"][0]
            kernel_name = "agg_insert+part_direct"
    avg_ms = ins_ms / max(1, ins_n)
    # algorithmic bytes of one insert launch
    keys_h = aggs_h = None
    if world == 1:
        n_groups = runner.n_groups
        kstr = runner.key_string_bytes
    else:
        runner.insert(0)  # (untimed) this rank's partial of copy 0, for the byte accounting
        n_groups = runner.table.finalize()[0]
        kstr = 0
        keys_h, aggs_h = None, None
    # selected rows: SUM of COUNT(*) over the partial table of this rank
    sel = None
    ci_star = next((i for i, (f, c) in enumerate(shape.aggs) if f == "count" and c is None), None)
    if world == 1 and ci_star is not None:  # on device: the result columns stay in HBM
        sel = int(runner.out_aggs[ci_star].data[: 8 * n_groups].view(torch.int64).sum().item())
    if sel is None:
        blk = runner.table.merge_result()
        ci = [i for i, (f, c) in enumerate(shape.aggs) if f == "count" and c is None]
        sel = int(sum(blk.columns[ci[0]].values())) if ci else rows
    alg_bytes = algorithmic_bytes(cfg, runner.inputs[0], rows, sel, n_groups, runner.result_types, kstr)
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0

    value = rows * world * args.steps / elapsed
    out = {
        "metric": "input rows/sec aggregated (filter + hash GROUP BY), % HBM roofline",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int16 key / u64 count" if cfg == 2 else "int64/decimal128/u64",
        "data": "synthetic (device-generated, seeded splitmix64; SURVEY.md §8d)",
        "config": {"workload": shape.name + ("" if scaling == "weak" or world == 1 else f"_strong_{total_rows}_rows"),
                   "query": shape.sql, "rows_per_gpu": rows, "input_copies": copies,
                   "groups": n_groups, "selected_rows": sel, "parallelism": f"dp{world}" if world > 1 else "single",
                   "strategy": "partitioned" if partitioned else "hbm_table",
                   "exchange": (("before_partial" if before_partial else "before_merge") + "/" + args.exchange)
                   if world > 1 and not small else ("replicas+gather" if world > 1 else None)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": kernel_name, "kernel_avg_ms": avg_ms, "kernel_launches": ins_n,
                     "algorithmic_bytes_per_launch": alg_bytes},
        "kernels_ms_per_step": {k: v[0] / args.steps for k, v in prof.items()},
    }
    # measured PMC traffic (rocprofv3 --pmc, committed under profiles/) if present for this config
    traffic, tsrc = load_traffic(cfg)
    if traffic:
        out["roofline"]["traffic"] = traffic
        out["roofline"]["traffic_source"] = tsrc
    # The ORDER BY <count> DESC LIMIT 10 that ends the ClickBench query, on the device result
    # (untimed leg, reported beside the step; dbg_sort_limit_indices).
    if world == 1 and n_groups > 0:
        ci_cnt = ci_star
        if ci_cnt is not None:
            from databend_amd.sort import sort_limit_indices
            dc = runner.out_aggs[ci_cnt]
            sort_limit_indices(dc, False, False, 10)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                idx = sort_limit_indices(dc, False, False, 10)
            torch.cuda.synchronize()
            sort_ms = (time.perf_counter() - t0) / 5 * 1e3
            counts = dc.data[: 8 * n_groups].view(torch.int64)  # check against torch's device top-k
            top = counts[idx.long()].tolist()
            ok = top == torch.topk(counts, min(10, n_groups)).values.tolist()
            out["order_by_limit"] = {"sql": "ORDER BY count DESC LIMIT 10", "ms": sort_ms, "groups": n_groups,
                                     "values_match_host_sort": ok}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample = args.cpu_sample_rows or {1: 6_001_215, 2: 100_000_000, 3: 20_000_000, 4: 10_000_000, 5: 20_000_000}[cfg]
        sample = min(sample, rows)
        cb, cres, _ = cpu_baseline(cfg, sample)
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "label", "sample", "sample_groups")}
        out["cpu_baseline"]["full_config_groups"] = n_groups
        out["gpu_vs_cpu"] = value / cb["value"]
        # parity of this bench's own GPU result against the CPU run when they cover the same rows
        if sample == rows and copies >= 1:
            try:
                from tests.parity import assert_results_equal
                runner.step(0)  # copy 0 == rows [0, rows) == the CPU sample
                kh, ah = runner.results_host()
                assert_results_equal(kh, ah, cres[0], cres[1])
                out["parity_vs_cpu"] = "bit-exact"
            except AssertionError as e:
                out["parity_vs_cpu"] = f"MISMATCH: {e}"
    # the other configurations of BASELINE.json, each at full size on this GPU, in the same run
    extra = args.extra_configs
    if extra is None:
        extra = "1,3,4,5" if (world == 1 and cfg == 2 and not args.rows) else "none"
    if world == 1 and extra != "none":
        runner.close()
        del runner
        torch.cuda.empty_cache()
        out["configs"] = {}
        for c in [int(x) for x in extra.split(",") if x.strip()]:
            if c == cfg:
                continue
            try:
                out["configs"][f"C{c}"] = measure_extra(c, args.extra_steps, 1, not args.no_cpu_baseline)
            except Exception as e:  # reported, never hidden: the headline line still prints
                out["configs"][f"C{c}"] = {"error": f"{type(e).__name__}: {e}"}
            print(f"bench.py: C{c} done", file=sys.stderr, flush=True)
        if extra == "1,3,4,5":  # the scan side beside the configurations
            try:
                out["scan"] = measure_scan(args.extra_steps + 2)
            except Exception as e:
                out["scan"] = {"error": f"{type(e).__name__}: {e}"}
            print("bench.py: scan done", file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure_scan(steps: int, rows: int = 1 << 26) -> dict:
    """Parquet -> HBM decode of C2's column as a Fuse block stores it (blocks_to_parquet: one row
    group — 2^26 rows, pyarrow's row-group cap — PLAIN, no dictionary, 1 MiB pages, Int16 stored as
    INT32 as arrow writers do; parquet_rs.rs:30-57), chunk bytes already resident in
    HBM: dbg_parquet_decode per chunk (host page-header parse + the device decode + one read-back),
    timed with events on the default stream.  Algorithmic bytes = the chunk's bytes read + the
    column's bytes written (values and validity)."""
    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pq
    import io
    import torch
    import ctypes as C
    from databend_amd import abi
    from databend_amd import column as col
    from databend_amd.ffi import check, lib
    from databend_amd.scan import ParquetChunkDecoder
    rng = np.random.default_rng(0xC2)
    adv = np.where(rng.random(rows) < 0.9937, 0, rng.integers(1, 33, rows)).astype(np.int16)
    res = {"workload": "clickbench AdvEngineID (Int16) column, 2^26 rows (one row group), Fuse parquet shape", "rows": rows}
    dec = ParquetChunkDecoder()
    for comp in ("NONE", "SNAPPY", "ZSTD"):
        t = pa.table({"a": pa.array(adv)}, schema=pa.schema([pa.field("a", pa.int16(), nullable=False)]))
        bio = io.BytesIO()
        pq.write_table(t, bio, compression=comp, use_dictionary=False, row_group_size=1 << 30, data_page_size=1 << 20)
        buf = bio.getvalue()
        md = pq.ParquetFile(io.BytesIO(buf)).metadata.row_group(0).column(0)
        chunk = buf[md.data_page_offset:md.data_page_offset + md.total_compressed_size]
        dchunk = torch.from_numpy(np.frombuffer(chunk, dtype=np.uint8).copy()).cuda()
        hbuf = C.create_string_buffer(chunk, len(chunk))
        c = abi.dbg_parquet_chunk()
        c.host = C.cast(hbuf, C.c_void_p)
        c.device = dchunk.data_ptr()
        c.len = len(chunk)
        c.physical_type = abi.PQ_INT32
        c.max_def_level = 0
        c.codec = {"NONE": abi.PQ_UNCOMPRESSED, "SNAPPY": abi.PQ_SNAPPY, "ZSTD": abi.PQ_ZSTD}[comp]
        out_t = torch.empty(rows * 2, dtype=torch.uint8, device="cuda")
        o = abi.dbg_out_column()
        o.data = out_t.data_ptr()
        nr, sb = C.c_uint64(), C.c_uint64()
        call = lambda: check(lib().dbg_parquet_decode(dec.h, C.byref(c), col.Int16.to_abi(), C.byref(o), rows, 0,
                                                     C.byref(nr), C.byref(sb)))
        call()
        assert nr.value == rows and torch.equal(out_t.view(torch.int16), torch.from_numpy(adv).cuda())
        from databend_amd import ffi
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ffi.prof_reset()
        ffi.prof_enable(True)
        ev0.record()
        for _ in range(steps):
            call()
        ev1.record()
        torch.cuda.synchronize()
        ffi.prof_enable(False)
        kern = ffi.prof_read()
        ms = ev0.elapsed_time(ev1) / steps
        alg = len(chunk) + rows * 2
        # device time of the decode kernels alone (HIP events on the decoder's stream): the rest of
        # ms_per_chunk is the host's page-header parse (one Thrift header per 20 000-row page) and the
        # call's launches / read-back
        kms = sum(v[0] for k, v in kern.items() if k in ("pq_decode", "pq_inflate")) / steps
        npg, nrw = C.c_uint32(), C.c_uint64()
        check(lib().dbg_parquet_chunk_rows(C.byref(c), C.byref(nrw), C.byref(npg)))
        res[comp.lower()] = {"chunk_bytes": len(chunk), "pages": npg.value,
                             "ms_per_chunk": ms, "rows_per_s": rows / (ms * 1e-3),
                             "achieved_gbs": alg / (ms * 1e-3) / 1e9, "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "kernel_ms_per_chunk": kms,
                             "kernel_frac": (alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS) if kms else None,
                             "algorithmic_bytes": alg, "bit_exact": True}
        del dchunk, out_t
    res.update(measure_native(dec, adv, steps))
    dec.close()
    return res


def native_pages(v, codec: str, page_rows: int = 131072):
    """The same column as Fuse's native format writes it (NativeWriter, 131072-row pages,
    non-nullable): 'dict_rle' is what choose_compressor picks for this column (Dict, its u32
    indices Rle-encoded: integer/dict.rs, rle.rs), 'lz4' / 'none' the basic codecs.  Synthetic
    bytes built with numpy here (bench input, not the oracle)."""
    import struct
    import numpy as np
    import pyarrow as pa
    out, lens, rows = bytearray(), [], []
    w = v.dtype.itemsize
    for s0 in range(0, len(v), page_rows):
        pv = v[s0:s0 + page_rows]
        n = len(pv)
        if codec == "dict_rle":
            u, first, inv = np.unique(pv, return_index=True, return_inverse=True)
            order = np.argsort(first, kind="stable")
            rank = np.empty(len(u), np.uint32)
            rank[order] = np.arange(len(u), dtype=np.uint32)
            idx = rank[inv.reshape(-1)]
            starts = np.concatenate([[0], np.flatnonzero(np.diff(idx)) + 1])
            runs = np.empty(len(starts), dtype=[("c", "<u4"), ("v", "<u4")])
            runs["c"] = np.diff(np.concatenate([starts, [n]]))
            runs["v"] = idx[starts]
            rb = runs.tobytes()
            inner = struct.pack("<BII", 10, len(rb), 4 * n) + rb
            payload = inner + struct.pack("<I", len(u)) + u[order].astype(v.dtype.newbyteorder("<")).tobytes()
            page = struct.pack("<BII", 11, len(payload), w * n) + payload
        else:
            raw = pv.astype(v.dtype.newbyteorder("<")).tobytes()
            body = pa.Codec("lz4_raw").compress(raw, asbytes=True) if codec == "lz4" else raw
            page = struct.pack("<BII", 1 if codec == "lz4" else 0, len(body), len(raw)) + body
        out += page
        lens.append(len(page))
        rows.append(n)
    return bytes(out), lens, rows


def measure_native(dec, adv, steps: int) -> dict:
    """Native (strawboat) pages of the same column -> HBM: dbg_native_decode per column, bytes
    resident in HBM, timed like the Parquet legs (host page walk + device decode + read-back)."""
    import numpy as np
    import torch
    import ctypes as C
    from databend_amd import abi
    from databend_amd import column as col
    from databend_amd import ffi
    from databend_amd.ffi import check, lib
    rows = len(adv)
    res = {}
    for codec in ("dict_rle", "lz4", "none"):
        buf, lens, prow = native_pages(adv, codec)
        dbuf = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy()).cuda()
        hbuf = C.create_string_buffer(buf, len(buf))
        hl = (C.c_uint64 * len(lens))(*lens)
        hr = (C.c_uint64 * len(prow))(*prow)
        c = abi.dbg_native_column()
        c.host = C.cast(hbuf, C.c_void_p)
        c.device = dbuf.data_ptr()
        c.len = len(buf)
        c.page_lengths = hl
        c.page_rows = hr
        c.n_pages = len(lens)
        c.nullable = 0
        out_t = torch.empty(rows * 2, dtype=torch.uint8, device="cuda")
        o = abi.dbg_out_column()
        o.data = out_t.data_ptr()
        nr, sb = C.c_uint64(), C.c_uint64()
        call = lambda: check(lib().dbg_native_decode(dec.h, C.byref(c), col.Int16.to_abi(), C.byref(o), rows, 0, C.byref(nr),
                                                    C.byref(sb)))
        call()
        assert nr.value == rows and torch.equal(out_t.view(torch.int16), torch.from_numpy(adv).cuda())
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ffi.prof_reset()
        ffi.prof_enable(True)
        ev0.record()
        for _ in range(steps):
            call()
        ev1.record()
        torch.cuda.synchronize()
        ffi.prof_enable(False)
        kern = ffi.prof_read()
        ms = ev0.elapsed_time(ev1) / steps
        kms = sum(v[0] for k, v in kern.items() if k in ("nat_decode", "nat_inflate")) / steps
        alg = len(buf) + rows * 2
        res["native_" + codec] = {"column_bytes": len(buf), "pages": len(lens), "ms_per_column": ms,
                                  "rows_per_s": rows / (ms * 1e-3), "achieved_gbs": alg / (ms * 1e-3) / 1e9,
                                  "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernel_ms_per_column": kms,
                                  "kernel_frac": (alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS) if kms else None,
                                  "algorithmic_bytes": alg, "bit_exact": True}
        del dbuf, out_t
    return res


if __name__ == "__main__":
    main()
