"""Rounds-to-target distributions of the reference [C] workload (real income CSV, compat mode:
overlapping seeded shards, local-shard evaluation, mean of client metrics, patience-10 /
atol-1e-4 early stop; FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:168-192).

For every (backend, dtype, k, seed) the k clients run in one process (fedmi/fl/simulate.py)
and the first round reaching 0.80 / 0.83 global accuracy, the early-stop round and the final
accuracy are recorded; a summary table (min / median / max per k) is printed next to the
reference's measured runs.

    python tools/rounds_to_target.py --backend torch --jobs 8 --out profiles/rtt_torch_r2.json
    python tools/rounds_to_target.py --backend hip --dtype fp32 bf16 --out profiles/rtt_hip_r2.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# BASELINE.md (reference, 3 unseeded runs per k)
REFERENCE = {
    1: {"0.80": [19, 19, 19], "0.83": [56, 80, 78], "early_stop_round": [216, 190, 203]},
    2: {"0.80": [27, 26, 23], "0.83": [130, 87, 64], "early_stop_round": [196, 169, 171]},
    4: {"0.80": [28, 30, 28], "0.83": [60, None, 91], "early_stop_round": [243, 164, 198]},
    8: {"0.80": [30, 29, 28], "0.83": [None, 121, 58], "early_stop_round": [162, 149, 194]},
}


def _one(args):
    backend, dtype, k, seed, max_rounds = args
    import torch
    if backend == "torch":
        torch.set_num_threads(1)
    from fedmi.data.tabular import load_tabular
    from fedmi.fl.engine import EngineConfig
    from fedmi.fl.simulate import rounds_to_target
    ds = load_tabular()
    cfg = EngineConfig(max_rounds=max_rounds, dtype=dtype)
    r = rounds_to_target(ds.X_train, ds.y_train, k, cfg, backend=backend, seed=seed)
    r.update(backend=backend, dtype=dtype, k=k, seed=seed)
    return r


def _fmt(vals):
    got = [v for v in vals if v is not None]
    never = len(vals) - len(got)
    if not got:
        return "never"
    s = f"{min(got)}/{int(np.median(got))}/{max(got)}"
    return s + (f" (+{never} never)" if never else "")


def summarize(rows):
    lines = ["| backend | dtype | k | runs | rounds to 0.80 (min/med/max) | rounds to 0.83 | early-stop round | "
             "final acc (mean) | reference stop rounds |", "|---|---|---|---|---|---|---|---|---|"]
    keys = sorted({(r["backend"], r["dtype"], r["k"]) for r in rows})
    for b, d, k in keys:
        rs = [r for r in rows if (r["backend"], r["dtype"], r["k"]) == (b, d, k)]
        ref = REFERENCE.get(k, {})
        lines.append(f"| {b} | {d} | {k} | {len(rs)} | {_fmt([r['0.80'] for r in rs])} | "
                     f"{_fmt([r['0.83'] for r in rs])} | {_fmt([r['early_stop_round'] for r in rs])} | "
                     f"{np.mean([r['final_acc'] for r in rs]):.4f} | {ref.get('early_stop_round')} |")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--dtype", nargs="+", default=["fp32"])
    ap.add_argument("--k", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--seeds", type=int, default=10)
    ap.add_argument("--max-rounds", type=int, default=300)
    ap.add_argument("--jobs", type=int, default=1, help="worker processes (torch backend)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dtypes = a.dtype if a.backend == "hip" else ["fp32"]
    work = [(a.backend, d, k, s, a.max_rounds) for d in dtypes for k in a.k for s in range(a.seeds)]
    rows = []
    if a.jobs > 1:
        with ProcessPoolExecutor(a.jobs) as ex:
            for r in ex.map(_one, work):
                rows.append(r)
                print(json.dumps(r), flush=True)
    else:
        for w in work:
            r = _one(w)
            rows.append(r)
            print(json.dumps(r), flush=True)
    table = summarize(rows)
    print(table, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "table": table, "reference": REFERENCE}, f, indent=1)


if __name__ == "__main__":
    main()
