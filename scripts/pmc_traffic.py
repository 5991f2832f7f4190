"""HBM traffic per launch of the dominant kernel from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; separate runs), corrected as MI355X_MICROARCH.md § HBM prescribes:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts wide coalesced streaming reads
at exactly half their bytes, so it is doubled.  Writes are taken as reported.

    python scripts/pmc_traffic.py gpurun_out/pmc_c2 agg_insert profiles/pmc_traffic_c2.json
"""
import csv
import json
import os
import sys


def per_launch(path, counter, kernel):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or kernel not in r["Kernel_Name"]:
            continue
        # one row per dispatch per counter instance (already summed by rocprofv3 for *_SIZE)
        vals.setdefault(r["Dispatch_Id"], 0.0)
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = list(vals.values())
    return sum(v) / len(v) if v else None, len(v), next(
        (r["Kernel_Name"] for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]), None)


def main():
    d, kernel, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch_kib, nf, kname = per_launch(os.path.join(d, "fetch_counter_collection.csv"), "FETCH_SIZE", kernel)
    write_kib, nw, _ = per_launch(os.path.join(d, "write_counter_collection.csv"), "WRITE_SIZE", kernel)
    read_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    res = {
        "kernel": kname,
        "launches": {"fetch_pass": nf, "write_pass": nw},
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "hbm_read_bytes_per_launch": read_b,
        "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "correction": "FETCH_SIZE x2 (gfx950 counts 16 B/lane streaming reads at half their bytes), KiB -> bytes; "
                      "WRITE_SIZE as reported (MI355X_MICROARCH.md, HBM section)",
        "source": os.path.relpath(d),
    }
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
