"""Driver-shaped timed region: one graph replay vs the same rounds issued eagerly from C++.

bench.py times `--steps 20` rounds as ONE replay of a 20-round graph; rocprofv3 with the HIP
runtime trace puts ~15 us between the `hipGraphLaunch` call and the first kernel
(profiles/graph_launch_lead_r5.log).  This tool builds bench.py's one-client engine (8000
rows, bf16, early-stop rule live) and alternates, per repetition:

  graph  prime a g-round graph, then time one replay (what bench.py does)
  eager  time FLEngine::run(r0, g) -- the same 2 g kernels, launched one by one from C++

Each region is bracketed exactly like bench.py (synchronize, perf_counter, ..., synchronize).

    python tools/eager_region.py [--rounds 20] [--reps 6]
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
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import numpy as np
    import torch
    from bench import synth_shard
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat

    dev = torch.device("cuda", 0)
    X, y = synth_shard(a.rows, 0, dev)
    g = a.rounds
    total = 5 + a.reps * (3 * g + 8) + 16  # per rep: prime (<= g + 4 eager + g replayed) + g timed + g eager
    cfg = EngineConfig(hidden=(50, 200), max_rounds=total, early_stop=True, patience=total + 1,
                       graph_rounds=g, dtype="bf16")
    stream = torch.cuda.Stream(device=dev)
    eng = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], seed=0), n_total=a.rows, stream=stream)
    eng.run(5, check_every=5)
    s = eng._stream()
    res = {"graph": [], "eager": []}
    for rep in range(a.reps):
        for mode in ("graph", "eager"):
            if mode == "graph":
                eng.prime_graph(g, replays=1)
            eng.stream.synchronize()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            if mode == "graph":
                eng._issue(g, close=False)
            else:
                eng.engine.run(eng.rounds_issued, g, s, eng._native_comm, False)
                eng.rounds_issued += g
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            res[mode].append(dt / g * 1e6)
            print(f"rep {rep} {mode:5s} {dt / g * 1e6:6.2f} us/round", flush=True)
    eng._issue(1)
    eng.sync_history()
    h = eng.history()
    assert h["stop_round"] < 0
    for k, v in res.items():
        print(f"{k:5s} median {np.median(v):6.2f}  min {min(v):6.2f}  max {max(v):6.2f} us/round over {len(v)} regions")


if __name__ == "__main__":
    main()
