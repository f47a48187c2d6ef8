"""Would a multi-client round be shorter if the previous round's local model were scored by the
evaluation kernel on a side stream, concurrently with the training kernel (a graph fork/join),
instead of by scoring waves inside the lagged training kernel?  Timing only (the kernels are
re-run on one live state; nothing is checked): per round, graph-replayed,

  plain       train + Adam                              (no scoring at all: the floor)
  lagged      lagged train kernel (register scoring) + Adam   (the current N > 1 round)
  serial      train + eval + Adam on one stream
  side        fork: eval on a side stream | train ; join; Adam

    python tools/probes/side_eval_probe.py [--rows 1000 2000 4000 8000] [--rounds 40] [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[1000, 2000, 4000, 8000])
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for rows in a.rows:
        X, y = bench.synth_shard(rows, 0, dev)
        cfg = EngineConfig(max_rounds=100000, early_stop=False, graph_rounds=0, dtype="bf16", fused_eval=False)
        e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, 50, 200, 2], 0), emulate_clients=True)
        e.run(4)
        r = e.rounds_issued - 1
        s = torch.cuda.Stream(device=dev)
        s2 = torch.cuda.Stream(device=dev)
        eng = e.engine

        def plain():
            eng.launch_one(r, 0, s.cuda_stream)
            eng.launch_one(r, 1, s.cuda_stream)

        def lagged():
            eng.launch_one(r, 3, s.cuda_stream)
            eng.launch_one(r, 1, s.cuda_stream)

        def serial():
            eng.launch_one(r, 0, s.cuda_stream)
            eng.launch_one(r, 2, s.cuda_stream)
            eng.launch_one(r, 1, s.cuda_stream)

        def side():
            fork = torch.cuda.Event()
            fork.record(s)
            s2.wait_event(fork)
            eng.launch_one(r, 2, s2.cuda_stream)
            eng.launch_one(r, 0, s.cuda_stream)
            join = torch.cuda.Event()
            join.record(s2)
            s.wait_event(join)
            eng.launch_one(r, 1, s.cuda_stream)

        res = {}
        for name, body in (("plain", plain), ("lagged", lagged), ("serial", serial), ("side", side)):
            s.wait_stream(torch.cuda.current_stream(dev))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.rounds):
                    body()
            g.replay()
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                with torch.cuda.stream(s):
                    g.replay()
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / a.rounds)
            res[name] = float(np.median(ts))
            del g
        print(f"rows {rows:5d} R={e.R}: " + "  ".join(f"{k} {v:6.2f}" for k, v in res.items()) + "  us/round",
              flush=True)
        del e


if __name__ == "__main__":
    main()
