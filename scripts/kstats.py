"""Short per-kernel summary of a rocprofv3 --stats kernel_stats.csv (long template names trimmed)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "rocprim" in n:
        tag = "histogram" if "histogram" in n else "iteration" if "iteration" in n else "transform" if "transform" in n else "other"
        n = "rocprim:" + tag
    print(f"{n[:70]:72s} calls={r['Calls']:>4} avg_us={float(r['AverageNs']) / 1e3:10.1f} total_ms={float(r['TotalDurationNs']) / 1e6:9.2f}")
