"""One config's steps delimited by profiler markers, for rocprofv3 counter passes.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c4/fetch -o fetch -- python scripts/pmc_run.py --config 4 --steps 2

Setup (data generation, table creation) and one warm-up step run first; then dbg_prof_marker,
`--steps` steps of the bench's runner (reset -> fused filter + GROUP BY -> finalize into HBM
result columns), dbg_prof_marker.  scripts/pmc_step_traffic.py attributes every dispatch between
the two markers to the steps.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, required=True)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--rows", type=int, default=0)
    a = p.parse_args()
    import torch
    from databend_amd.ffi import check, lib
    from databend_amd.workloads import DEFAULT_ROWS, ConfigRunner
    rows = a.rows or DEFAULT_ROWS[a.config]
    r = ConfigRunner(a.config, rows, copies=1)
    r.step(0)
    torch.cuda.synchronize()
    check(lib().dbg_prof_marker(torch.cuda.current_stream().cuda_stream))
    for k in range(a.steps):
        r.step(1 + k)
    check(lib().dbg_prof_marker(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    print(f"pmc_run: config {a.config}, {rows} rows, {a.steps} steps, {r.n_groups} groups", flush=True)
    r.close()


if __name__ == "__main__":
    main()
