"""FETCH_SIZE / WRITE_SIZE calibration (scripts/micro/fetch_calib.hip) on gfx950: the counter of
each measured (second) dispatch divided by the bytes it moves or the distinct 64-B lines it
touches.  MI355X_MICROARCH.md calibrates only 16 B/lane streaming reads (FETCH_SIZE = half);
this covers the 8-B streaming and the random 8/16-B probe, 8-B atomic and 16-B store shapes of
this repo's kernels.

    python scripts/pmc_calib.py <fetch dir> <write dir> <fetch_calib stdout json> <out json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ["stream16", "stream8", "rand_load<8>", "rand_load<16>", "rand_atom8", "rand_store16", "stream_store16"]


def per_dispatch(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        disp[k] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    out = defaultdict(list)
    for k in sorted(disp):
        n = names[k]
        n = n[5:] if n.startswith("void ") else n
        base = n.split("(")[0].replace(" ", "")
        if base in KERNELS:
            out[base].append(disp[k] * 1024.0)  # KiB -> bytes
    return {k: v[-1] for k, v in out.items()}  # the second (measured) dispatch


def main():
    fdir, wdir, known_path, out_path = sys.argv[1:5]
    known = json.loads(open(known_path).read().strip().splitlines()[-1])
    f = per_dispatch(fdir, "FETCH_SIZE")
    w = per_dispatch(wdir, "WRITE_SIZE")
    B, ops, dl = known["buffer_bytes"], known["random_ops"], known["distinct_lines"]
    res = {
        "stream16_read": {"bytes": B, "fetch_size": f.get("stream16"), "fetch_over_bytes": f.get("stream16", 0) / B},
        "stream8_read": {"bytes": B, "fetch_size": f.get("stream8"), "fetch_over_bytes": f.get("stream8", 0) / B},
        "rand8_read": {"loads": ops, "distinct_lines": dl["rand_load8"], "fetch_size": f.get("rand_load<8>"),
                       "fetch_per_line": f.get("rand_load<8>", 0) / dl["rand_load8"]},
        "rand16_read": {"loads": ops, "distinct_lines": dl["rand_load16"], "fetch_size": f.get("rand_load<16>"),
                        "fetch_per_line": f.get("rand_load<16>", 0) / dl["rand_load16"]},
        "rand8_atomic": {"ops": ops, "distinct_lines": dl["rand_atom8"], "fetch_size": f.get("rand_atom8"),
                         "write_size": w.get("rand_atom8"),
                         "fetch_per_op": f.get("rand_atom8", 0) / ops, "write_per_op": w.get("rand_atom8", 0) / ops},
        "rand16_store": {"ops": ops, "distinct_lines": dl["rand_store16"], "write_size": w.get("rand_store16"),
                         "fetch_size": f.get("rand_store16"), "write_per_op": w.get("rand_store16", 0) / ops},
        "stream16_store": {"bytes": B, "write_size": w.get("stream_store16"),
                           "write_over_bytes": w.get("stream_store16", 0) / B},
        "source": {"fetch": os.path.relpath(fdir), "write": os.path.relpath(wdir)},
    }
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
