"""Per-kernel duration and launch gap statistics from a rocprofv3 kernel trace CSV.

usage: python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [name-filter]
Gap = start of a kernel - end of the previous kernel on the same queue (device idle time
between dependent kernels of the round)."""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
filt = sys.argv[2] if len(sys.argv) > 2 else "fl_"
rows = [r for r in rows if filt in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
gap_before = defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:48]
    dur[name].append(e - s)
    if prev_end is not None and s >= prev_end:
        gap_before[name].append(s - prev_end)
    prev_end = e
tot = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"{len(rows)} kernels over {tot:.1f} us")
for k in dur:
    d = np.array(dur[k]) / 1e3
    g = np.array(gap_before[k]) / 1e3 if gap_before[k] else np.zeros(1)
    print(f"{k:48s} n={len(d):6d} dur med {np.median(d):7.2f} p90 {np.percentile(d, 90):7.2f} us | "
          f"gap before med {np.median(g):6.2f} p90 {np.percentile(g, 90):6.2f} us")
