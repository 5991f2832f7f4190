"""Per-kernel LDS / atomic / occupancy counters of one step, from rocprofv3 --pmc passes over
scripts/pmc_run.py (one counter group per run; scripts/gpu_pmc_lds.sh), attributed to the
dispatches between the two dbg_marker_kernel dispatches (one step).

    python scripts/pmc_lds_summary.py gpurun_out/pmclds_c4 STEPS profiles/pmc_lds_atomics_c4.json

Derived figures (MI355X_MICROARCH.md "LDS" and "rocprofv3 PMC slots"):
  bank_conflict_cycles_per_lds_inst = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra LDS cycles per
      wave-level LDS instruction; 0 = conflict-free)
  bank_conflict_frac_of_lds_active  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (share of the LDS
      array's busy cycles spent on conflicts)
  wait_inst_lds_frac                = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (waves stalled issuing LDS)
  wait_any_frac                     = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  lds_atomic_return_per_wave        = SQ_LDS_ATOMIC_RETURN / SQ_WAVES
  l2_atomics / mem_atomics          = TCC_ATOMIC_sum / TCC_EA0_ATOMIC_sum per step (memory-side
      atomics are the ones that leave the L2 for HBM: device-scope atomics on gfx950 with
      -munsafe-fp-atomics off the fp path)
Kernel resources (Scratch_Size bytes/lane, VGPR/SGPR counts, LDS bytes) come from the same CSV.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(path):
    """{dispatch: (name, {counter: value}, duration_ns, resources)} of every counter CSV under path."""
    disp = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            name = r["Kernel_Name"]
            e = disp.setdefault(k, [name, defaultdict(float), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                    {"scratch_bytes_per_lane": int(r["Scratch_Size"]), "vgpr": int(r["VGPR_Count"]),
                                     "agpr": int(r["Accum_VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                                     "lds_bytes": int(r["LDS_Block_Size"]), "workgroup": int(r["Workgroup_Size"])}])
            e[1][r["Counter_Name"]] += float(r["Counter_Value"])
    return disp


def step_kernels(disp):
    order = sorted(disp)
    marks = [k for k in order if "dbg_marker_kernel" in disp[k][0]]
    if len(marks) < 2:
        raise SystemExit(f"expected two dbg_marker_kernel dispatches, found {len(marks)}")
    a, b = marks[-2], marks[-1]
    return [disp[k] for k in order if a < k < b]


def main():
    root, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    kern = {}
    for pas in sorted(os.listdir(root)):
        d = os.path.join(root, pas)
        if not os.path.isdir(d):
            continue
        for name, ctr, dur, res in step_kernels(load(d)):
            e = kern.setdefault(name, {"launches_per_step": 0, "resources": res, "counters": defaultdict(float), "dur_ns": [],
                                       "_passes": defaultdict(int)})
            e["_passes"][pas] += 1
            e["dur_ns"].append(dur)
            for c, v in ctr.items():
                e["counters"][c] += v
    res = {}
    for name, e in kern.items():
        launches = max(e["_passes"].values()) / steps
        c = {k: v / steps for k, v in e["counters"].items()}
        r = {"launches_per_step": launches, "resources": e["resources"],
             "avg_duration_us_under_pmc": round(sum(e["dur_ns"]) / len(e["dur_ns"]) / 1e3, 3),
             "counters_per_step": {k: round(v, 1) for k, v in sorted(c.items())}}
        der = {}
        if c.get("SQ_INSTS_LDS"):
            der["bank_conflict_cycles_per_lds_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
        if c.get("SQ_LDS_IDX_ACTIVE"):
            der["bank_conflict_frac_of_lds_active"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("SQ_WAVE_CYCLES"):
            der["wait_inst_lds_frac"] = c.get("SQ_WAIT_INST_LDS", 0) / c["SQ_WAVE_CYCLES"]
            der["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_WAVES"):
            w = c["SQ_WAVES"]
            for k in ("SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_LDS_ATOMIC_RETURN"):
                if k in c:
                    der[k.lower().replace("sq_", "") + "_per_wave"] = c[k] / w
        if "TCC_ATOMIC_sum" in c:
            der["l2_atomics_per_step"] = c["TCC_ATOMIC_sum"]
        if "TCC_EA0_ATOMIC_sum" in c:
            der["mem_atomics_per_step"] = c["TCC_EA0_ATOMIC_sum"]
        r["derived"] = {k: round(v, 4) for k, v in der.items()}
        res[name] = r
    doc = {"scope": "one step (between the dbg_marker_kernel dispatches of scripts/pmc_run.py), per kernel, summed over "
                    "its launches in the step; one counter group per rocprofv3 run (scripts/gpu_pmc_lds.sh)",
           "steps": steps, "source": os.path.relpath(root),
           "kernels": dict(sorted(res.items(), key=lambda kv: -kv[1]["avg_duration_us_under_pmc"] * kv[1]["launches_per_step"]))}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(doc, open(out, "w"), indent=1)
    for name, r in list(doc["kernels"].items())[:10]:
        d = r["derived"]
        print(f"{name[:70]:72s} x{r['launches_per_step']:.0f} {r['avg_duration_us_under_pmc']:9.1f}us scratch={r['resources']['scratch_bytes_per_lane']} "
              f"vgpr={r['resources']['vgpr']} bank/lds={d.get('bank_conflict_cycles_per_lds_inst', 0):.3f} "
              f"waitlds={d.get('wait_inst_lds_frac', 0):.3f} l2at={d.get('l2_atomics_per_step', 0):.3g} memat={d.get('mem_atomics_per_step', 0):.3g}")


if __name__ == "__main__":
    main()
