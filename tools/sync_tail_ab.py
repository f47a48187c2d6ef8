"""A/B: how the driver-shaped timed region (one 20-round graph replay, one client, 8000 rows, bf16) waits for
the GPU.  profiles/graph_launch_lead_r5.log: hipDeviceSynchronize returns ~13 us after the last kernel ends.
Every variant ends with torch.cuda.synchronize() (the bench contract); they differ in what runs before it:

  device   torch.cuda.synchronize() alone (bench.py today)
  stream   engine-stream synchronize, then torch.cuda.synchronize()
  event    an event recorded behind the replay, event.synchronize(), then torch.cuda.synchronize()
  spin     busy-poll event.query(), then torch.cuda.synchronize()

    python tools/sync_tail_ab.py [--reps 15]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X, y = bench.synth_shard(8000, 0, dev)
    total = 5 + 4 * a.reps * a.steps + 200
    cfg = EngineConfig(max_rounds=total, early_stop=True, patience=total + 1, graph_rounds=a.steps, dtype="bf16")
    e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], 0), n_total=8000)
    e.run(5, check_every=5)
    e.prime_graph(a.steps)
    s = e._stream()
    ev = torch.cuda.Event()

    def wait(kind):
        if kind == "stream":
            e.stream.synchronize()
        elif kind == "event":
            ev.record(e.stream)
            ev.synchronize()
        elif kind == "spin":
            ev.record(e.stream)
            while not ev.query():
                pass
        torch.cuda.synchronize(dev)

    kinds = ("device", "stream", "event", "spin")
    res = {k: [] for k in kinds}
    for rep in range(a.reps):
        for k in kinds:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            e.engine.replay(s)
            wait(k)
            res[k].append((time.perf_counter() - t0) / a.steps * 1e6)
            e.rounds_issued += a.steps
    for k, v in res.items():
        v = np.asarray(v[1:])
        print(f"{k:7s}: us/round median {np.median(v):.2f}  min {v.min():.2f}  max {v.max():.2f}", flush=True)
    e._issue(1)
    e.sync_history()
    assert e.history()["stop_round"] < 0


if __name__ == "__main__":
    main()
