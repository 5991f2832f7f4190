"""Per-kernel summary of scripts/gpu_profile.sh output: kernel-trace stats plus the PMC passes
(SQ instruction / LDS counters, FETCH_SIZE, WRITE_SIZE, L2 atomics), per launch, with the
MI355X_MICROARCH.md corrections (FETCH_SIZE / WRITE_SIZE in KiB; FETCH_SIZE doubled for wide
coalesced streaming reads on gfx950).

    python scripts/pmc_summary.py gpurun_out/prof profiles/r02/pmc_all.json
"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    return n[:80]


def load_pmc(path):
    per = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            d = per.setdefault(k, {})
            disp = d.setdefault(r["Dispatch_Id"], {})
            disp[r["Counter_Name"]] = disp.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main():
    root, out = sys.argv[1], sys.argv[2]
    res = {"note": "rocprofv3 per-kernel: kernel-trace stats (bench steps) and PMC passes of one bench step after one "
                   "warm-up step, one counter group per run; *_per_launch = mean over the last step's dispatches; fetch_bytes = "
                   "FETCH_SIZE x 1024 x 2 (gfx950: wide streaming reads count half), write_bytes = WRITE_SIZE x 1024; "
                   "lds_bank_conflict_cycles_per_lds_inst = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS; "
                   "l2_atomics / mem_atomics = TCC_ATOMIC_sum / TCC_EA0_ATOMIC_sum per launch",
           "configs": {}}
    for cdir in sorted(glob.glob(os.path.join(root, "c[0-9]"))):
        cfg = os.path.basename(cdir)
        kern = {}
        for f in glob.glob(os.path.join(cdir, "stats", "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Name"])
                kern.setdefault(k, {})["calls"] = int(r["Calls"])
                kern[k]["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
                kern[k]["total_ms"] = round(float(r["TotalDurationNs"]) / 1e6, 3)
        for pas in ("sq", "fetch", "write", "atom"):
            per = load_pmc(os.path.join(cdir, pas))
            for k, disp in per.items():
                # the PMC runs are one warm-up step + one step: keep the last step's dispatches
                # (the later half by dispatch id), so first-batch table growth is not averaged in
                ids = sorted(disp, key=int)
                ids = ids[len(ids) // 2:] if len(ids) > 1 else ids
                n = len(ids)
                tot = {}
                for dv in (disp[i] for i in ids):
                    for c, v in dv.items():
                        tot[c] = tot.get(c, 0.0) + v
                e = kern.setdefault(k, {})
                for c, v in tot.items():
                    e[c + "_per_launch"] = v / n
        for k, e in kern.items():
            if "FETCH_SIZE_per_launch" in e:
                e["fetch_bytes_per_launch"] = e["FETCH_SIZE_per_launch"] * 1024 * 2
            if "WRITE_SIZE_per_launch" in e:
                e["write_bytes_per_launch"] = e["WRITE_SIZE_per_launch"] * 1024
            if e.get("SQ_INSTS_LDS_per_launch"):
                e["lds_bank_conflict_cycles_per_lds_inst"] = e.get("SQ_LDS_BANK_CONFLICT_per_launch", 0) / e["SQ_INSTS_LDS_per_launch"]
            if e.get("SQ_WAVE_CYCLES_per_launch"):
                e["wait_lds_frac"] = e.get("SQ_WAIT_INST_LDS_per_launch", 0) / e["SQ_WAVE_CYCLES_per_launch"]
            for c in list(e):
                if isinstance(e[c], float):
                    e[c] = round(e[c], 4)
        res["configs"][cfg] = kern
    json.dump(res, open(out, "w"), indent=1)
    for cfg, kern in res["configs"].items():
        print(cfg)
        for k, e in sorted(kern.items(), key=lambda kv: -kv[1].get("total_ms", 0))[:8]:
            print(f"  {k[:50]:52s} avg_us={e.get('avg_us')} fetchMB={e.get('fetch_bytes_per_launch', 0)/1e6:.1f} "
                  f"writeMB={e.get('write_bytes_per_launch', 0)/1e6:.1f} bankc/lds={e.get('lds_bank_conflict_cycles_per_lds_inst', 0):.2f} "
                  f"l2atom={e.get('TCC_ATOMIC_sum_per_launch', 0):.0f} memAtom={e.get('TCC_EA0_ATOMIC_sum_per_launch', 0):.0f}")


if __name__ == "__main__":
    main()
