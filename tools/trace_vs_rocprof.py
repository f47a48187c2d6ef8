"""Compare FLEngine::trace intervals with rocprofv3 kernel durations of the same run.

Reads a rocprofv3 database (``--kernel-trace`` output, rocpd sqlite) of a ``bench.py`` run
and prints, for the rounds traced after the timed region (the dispatches after the
``fl_gate_kernel``; its first ``--warm`` rounds untraced), each kernel's mean device
duration and start-to-start spacing, plus the same for the timed region's graph-replay
rounds (the gap-free run of dispatches before the gate).

    python tools/trace_vs_rocprof.py gpurun_out/.../run_results.db [--warm 2 --rounds 8]
"""
import argparse
import sqlite3
import statistics as st


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    gate = [i for i, r in enumerate(rows) if "fl_gate_kernel" in r[0]]
    if not gate:
        raise SystemExit("no fl_gate_kernel dispatch in the trace")
    g = gate[0]
    short = lambda n: n.split("(")[0].split("<")[0].replace("void ", "")
    per = 2  # train + adam per traced round (one client, fused rounds)
    traced = rows[g + 1 + per * a.warm: g + 1 + per * (a.warm + a.rounds)]
    # the timed region: the contiguous graph-replay dispatches (no host gap > 20 us) before the gate
    i = g - 1
    while i > 0 and rows[i][1] - rows[i - 1][2] < 20_000 and g - i < 400:
        i -= 1
    steady = rows[i:g]
    if "train" not in steady[0][0]:
        steady = steady[1:]
    steady = steady[: len(steady) // per * per]

    def summary(tag, seq):
        by = {}
        for i, (n, s, e) in enumerate(seq):
            nxt = seq[i + 1][1] if i + 1 < len(seq) else None
            d = by.setdefault(short(n), {"dur": [], "gap": []})
            d["dur"].append((e - s) / 1e3)
            if nxt is not None:
                d["gap"].append((nxt - s) / 1e3)
        for k, d in by.items():
            print(f"{tag:8s} {k:32s} n={len(d['dur']):3d} duration {st.mean(d['dur']):7.2f} us  "
                  f"start-to-next-start {st.mean(d['gap']) if d['gap'] else float('nan'):7.2f} us")
        span = (seq[-1][2] - seq[0][1]) / 1e3
        print(f"{tag:8s} span {span:.1f} us over {len(seq) // per} rounds = {span / (len(seq) // per):.2f} us/round")

    summary("steady", steady)
    summary("traced", traced)


if __name__ == "__main__":
    main()
