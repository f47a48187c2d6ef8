"""A/B: the driver-shaped timed region (bench.py --steps 20 --warmup 5, one client, 8000 rows, bf16,
early-stop rule live) as ONE 20-round graph replay vs a short LEAD graph followed by the rest.

profiles/graph_launch_lead_r5.log: the first kernel of a 20-round graph starts ~15 us after
hipGraphLaunch, and hipGraphLaunch keeps submitting the graph's 40 packets for ~320 us while the
GPU runs them.  If the lead grows with the graph's node count, a 2-round lead graph starts the GPU
sooner and the second launch is issued while the first graph runs.  Every variant times exactly
the same 20 rounds with bench.py's bracket (synchronize, t0, replays, synchronize, t1), interleaved.

    python tools/split_launch_ab.py [--reps 12] [--steps 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8000)
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--splits", nargs="+", default=["20", "e2,18", "e1,e1,18", "e4,16", "2,18"],
                    help="comma-separated parts; 'eN' = N rounds launched eagerly (no graph)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, y = bench.synth_shard(a.rows, 0, dev)
    total = 5 + a.reps * a.steps + 200
    stream = torch.cuda.Stream(device=dev)
    variants = {}
    for sp in a.splits:
        parts = sp.split(",")
        n = [int(x.lstrip("e")) for x in parts]
        assert sum(n) == a.steps and all(int(x) % 2 == 0 for x in parts if not x.startswith("e")), sp
        gsz = sorted({int(x) for x in parts if not x.startswith("e")})
        cfg = EngineConfig(max_rounds=total, early_stop=True, patience=total + 1, graph_rounds=gsz[-1],
                           dtype="bf16")
        e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], 0), n_total=a.rows, stream=stream)
        e.run(5, check_every=5)
        for g in gsz:                         # capture + instantiate + one replay of every graph size
            e.prime_graph(g)
        variants[sp] = (e, parts)
    s = stream.cuda_stream
    res = {sp: [] for sp in variants}
    for rep in range(a.reps):
        for sp, (e, parts) in variants.items():
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            r = e.rounds_issued
            for x in parts:
                if x.startswith("e"):           # eager launches from C++ (no graph)
                    e.engine.run(r, int(x[1:]), s, None, close=False)
                    r += int(x[1:])
                else:
                    e.engine.capture(int(x), s, None)    # selects the cached graph (no capture)
                    e.engine.replay(s)
                    r += int(x)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            e.rounds_issued += a.steps
            res[sp].append(dt / a.steps * 1e6)
    for sp, v in res.items():
        v = np.asarray(v[1:])   # first rep dropped (warm)
        print(f"split {sp:>8s}: us/round median {np.median(v):.2f}  min {v.min():.2f}  max {v.max():.2f}  "
              f"({len(v)} reps)", flush=True)
    for sp, (e, _) in variants.items():
        e._issue(1)
        e.sync_history()
        h = e.history()
        assert h["stop_round"] < 0, sp
    print("every timed round live (no early stop)", flush=True)


if __name__ == "__main__":
    main()
