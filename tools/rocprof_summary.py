"""Summaries of rocprofv3 CSV output for profiles/.

    python tools/rocprof_summary.py stats <dir>          # per-kernel time table (--kernel-trace --stats)
    python tools/rocprof_summary.py pmc <dir> [<dir>...] # per-kernel counter means (--pmc passes)

The PMC view prints raw counters per dispatch and, where the inputs were collected:
  * LDS bank-conflict cycles per LDS instruction (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS)
  * MFMA-busy share (SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES)
  * MFMA work (SQ_INSTS_VALU_MFMA_MOPS_*; 512 FLOP per MOP)
  * the wave-cycle split active / issue-stalled / parked (SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY,
    SQ_WAIT_ANY over SQ_WAVE_CYCLES)
gfx950 has no derived-counter XML in ROCm 7.2 (rocprofv3's derived metrics fall back to gfx94x
formulas), so only raw counters and these ratios are reported.
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def _find(d: str, suffix: str) -> list:
    return sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))


def stats(d: str) -> None:
    files = _find(d, "kernel_stats.csv")
    if not files:
        print(f"no kernel_stats.csv under {d}")
        return
    rows = list(csv.DictReader(open(files[0])))
    total = sum(float(x["TotalDurationNs"]) for x in rows)
    print(f"{'kernel':64s} {'calls':>7s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for x in rows:
        print(f"{x['Name'][:64]:64s} {int(x['Calls']):7d} {float(x['AverageNs']) / 1e3:9.2f} "
              f"{float(x['MinNs']) / 1e3:9.2f} {float(x['MaxNs']) / 1e3:9.2f} {float(x['Percentage']):6.2f}")
    print(f"total kernel time {total / 1e6:.3f} ms")


def pmc(dirs) -> None:
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for f in _find(d, "counter_collection.csv"):
            for x in csv.DictReader(open(f)):
                k = x.get("Kernel_Name") or x.get("Kernel-Name") or "?"
                k = k.split("(")[0][:60]
                name = x["Counter_Name"]
                acc[k][name] += float(x["Counter_Value"])
                disp[(k, name)].add((f, x.get("Dispatch_Id", "")))
    if not acc:
        print("no counter_collection.csv found")
        return
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        per = {name: v / max(1, len(disp[(k, name)])) for name, v in c.items()}
        n = max(len(disp[(k, name)]) for name in c)
        print(f"== {k}  ({n} dispatches per pass)")
        for name in sorted(per):
            print(f"   {name:32s} {per[name]:16.1f} per dispatch")
        if per.get("SQ_INSTS_LDS"):
            print(f"   -> LDS bank-conflict cycles per LDS instr: "
                  f"{per.get('SQ_LDS_BANK_CONFLICT', 0) / per['SQ_INSTS_LDS']:.3f}")
        if per.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in per:
            print(f"   -> MFMA busy cycles / SQ busy cycles: {per['SQ_VALU_MFMA_BUSY_CYCLES'] / per['SQ_BUSY_CYCLES']:.3f}")
        mops = per.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) + per.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0)
        if mops:
            print(f"   -> MFMA work per dispatch: {mops:.0f} MOPs = {mops * 512 / 1e9:.4f} GFLOP")
        w = per.get("SQ_WAVE_CYCLES")
        if w:
            parts = [(nm, per.get(nm, 0) / w) for nm in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")]
            if any(v for _, v in parts):
                print("   -> wave-cycle split: " + ", ".join(f"{nm[3:]} {v:.2f}" for nm, v in parts))


def main(argv) -> int:
    if len(argv) < 2:
        print(__doc__)
        return 2
    if argv[0] == "stats":
        stats(argv[1])
    elif argv[0] == "pmc":
        pmc(argv[1:])
    else:
        print(__doc__)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
