"""The bench's scan leg (bench.measure_scan) alone, for rocprofv3 --kernel-trace --stats: where a
dbg_parquet_decode call's time goes (device kernels vs host parse / copies / read-back)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

t0 = time.perf_counter()
r = bench.measure_scan(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
print(json.dumps(r))
print("wall s", time.perf_counter() - t0, file=sys.stderr)
