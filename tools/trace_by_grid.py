"""rocprofv3 kernel trace -> time per (kernel, grid, LDS, VGPRs): kernels that share a name but run
different shapes (trial batches of different hidden sizes, R = 32 vs 64 workgroups) separated,
plus the wall span of the traced region and the busy fraction (union of dispatch intervals).

    python tools/trace_by_grid.py gpurun_out/<dir>/run_kernel_trace.csv [--last N]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=0, help="only the last N dispatches (the steady region)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.last:
        rows = rows[-a.last:]
    agg = defaultdict(lambda: [0, 0.0])
    iv = []
    for r in rows:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv.append((t0, t1))
        gx = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        key = (r["Kernel_Name"].split("(")[0][:48], gx, int(r["Grid_Size_Y"]), int(r["Workgroup_Size_X"]),
               int(r["LDS_Block_Size"]), int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"]))
        agg[key][0] += 1
        agg[key][1] += (t1 - t0) / 1e3
    busy, cur0, cur1 = 0.0, None, None
    for t0, t1 in sorted(iv):
        if cur1 is None or t0 > cur1:
            if cur1 is not None:
                busy += cur1 - cur0
            cur0, cur1 = t0, t1
        else:
            cur1 = max(cur1, t1)
    if cur1 is not None:
        busy += cur1 - cur0
    span = (max(t for _, t in iv) - min(t for t, _ in iv)) / 1e3 if iv else 0.0
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':48s} {'wgs':>6s} {'y':>3s} {'thr':>5s} {'lds':>7s} {'vgpr':>5s} {'calls':>6s} {'avg_us':>8s} {'sum%':>6s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[0]:48s} {k[1]:6d} {k[2]:3d} {k[3]:5d} {k[4]:7d} {k[5]:5d} {n:6d} {t / n:8.2f} {100 * t / tot:6.2f}")
    print(f"span {span:.1f} us, busy (union of dispatches) {busy / 1e3:.1f} us = {100 * busy / 1e3 / max(span, 1e-9):.1f} %, "
          f"sum of kernel times {tot:.1f} us (overlap factor {tot / max(busy / 1e3, 1e-9):.2f})")


if __name__ == "__main__":
    main()
