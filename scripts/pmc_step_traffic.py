"""HBM traffic per step from two rocprofv3 --pmc passes over scripts/pmc_run.py (FETCH_SIZE and
WRITE_SIZE in separate runs), corrected as MI355X_MICROARCH.md's HBM section prescribes: the
counters are in KiB; on gfx950 FETCH_SIZE counts every 128-B read request (streaming or a random
probe's miss) as 64 B, so it is doubled; WRITE_SIZE is taken as reported (calibrated against known
bytes and the TCC_EA0_RDREQ/WRREQ request counters: profiles/r04/pmc_calibration.json).  Every dispatch between the two
dbg_marker_kernel dispatches belongs to the timed steps.

    python scripts/pmc_step_traffic.py gpurun_out/pmc_c4 STEPS profiles/pmc_traffic_c4.json [algorithmic_bytes]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _csv(d, stem):
    hits = glob.glob(os.path.join(d, "**", f"*{stem}*counter_collection.csv"), recursive=True)
    if not hits:
        raise SystemExit(f"no {stem} counter_collection.csv under {d}")
    return hits[0]


def per_step(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    disp = {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        name, v = r["Kernel_Name"], float(r["Counter_Value"])
        n0, v0 = disp.get(k, (name, 0.0))
        disp[k] = (name, v0 + v)
    order = sorted(disp)
    marks = [k for k in order if "dbg_marker_kernel" in disp[k][0]]
    if len(marks) < 2:
        raise SystemExit(f"{path}: expected two dbg_marker_kernel dispatches, found {len(marks)}")
    a, b = marks[-2], marks[-1]
    by_kernel = defaultdict(float)
    total = 0.0
    for k in order:
        if a < k < b:
            by_kernel[disp[k][0]] += disp[k][1]
            total += disp[k][1]
    return total, by_kernel


def main():
    d, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    f_kib, f_by = per_step(_csv(d, "fetch"), "FETCH_SIZE")
    w_kib, w_by = per_step(_csv(d, "write"), "WRITE_SIZE")
    read_b = 2.0 * f_kib * 1024.0 / steps
    write_b = w_kib * 1024.0 / steps
    # keyed by the FULL kernel name: template instantiations (and library kernels) share long
    # prefixes, and a truncated key let one overwrite another (round 3: rocPRIM's passes)
    kernels = {}
    for name in sorted(set(f_by) | set(w_by), key=lambda n: -(2 * f_by.get(n, 0) + w_by.get(n, 0))):
        kernels[name] = {"read": 2.0 * f_by.get(name, 0.0) * 1024.0 / steps, "write": w_by.get(name, 0.0) * 1024.0 / steps}
    attributed = sum(v["read"] + v["write"] for v in kernels.values())
    assert abs(attributed - (read_b + write_b)) <= 1e-6 * max(1.0, read_b + write_b), (attributed, read_b + write_b)
    res = {
        "scope": "every dispatch of one step (between dbg_marker_kernel dispatches of scripts/pmc_run.py)",
        "steps": steps,
        "hbm_read_bytes_per_step": read_b,
        "hbm_write_bytes_per_step": write_b,
        "hbm_bytes_per_step": read_b + write_b,
        "hbm_bytes_per_launch": read_b + write_b,  # bench.py reads this key (one step = one launch of C2's fused kernel)
        "algorithmic_bytes": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg if alg else None,
        "kernels_per_step": kernels,
        "correction": "FETCH_SIZE x2 (gfx950 counts each 128-B read request, streaming or random, as 64 B: "
                      "profiles/r04/pmc_calibration.json), KiB -> bytes; WRITE_SIZE as reported",
        "source": os.path.relpath(d),
    }
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels_per_step"}))


if __name__ == "__main__":
    main()
