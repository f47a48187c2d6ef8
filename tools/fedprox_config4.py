"""BASELINE config 4: 8 clients, Dirichlet label-skew shards (alpha 0.3), 5 local Adam steps per
round, 50 rounds, FedProx mu in {0, 0.01, 0.1}; held-out test metrics of the aggregated model.

The 8 clients run in one process (fedmi/fl/simulate.py): ``--backend hip`` on one GPU (fp32
classic rounds: train + Adam (FedProx term fused) + eval kernels per client, device-side
FedAvg), ``--backend torch`` the eager oracle on CPU.  Same shards (label_skew, seed 0) and the
same per-client inits as the one-process-per-client run of tools/fedprox_config4.sh.

    python tools/fedprox_config4.py --backend hip --out profiles/fedprox_config4_hip_r2.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--mu", type=float, nargs="+", default=[0.0, 0.01, 0.1])
    ap.add_argument("--alpha", type=float, default=0.3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    from fedmi.data.tabular import load_tabular
    from fedmi.fl.engine import EngineConfig
    from fedmi.fl.metrics import metrics_from_confusion
    from fedmi.fl.simulate import ClientGroup
    if a.backend == "torch":
        torch.set_num_threads(1)
    ds = load_tabular()
    res = []
    for mu in a.mu:
        cfg = EngineConfig(max_rounds=a.rounds, local_steps=5, prox_mu=mu, early_stop=False, dtype=a.dtype)
        g = ClientGroup(ds.X_train, ds.y_train, a.clients, cfg, backend=a.backend, shard_mode="label_skew",
                        alpha=a.alpha, seed=0)
        t0 = time.perf_counter()
        g.run(a.rounds)
        dt = time.perf_counter() - t0
        lead = g.clients[0]
        cm = lead.confusion(ds.X_test, ds.y_test, flat=g.global_flat())
        test = metrics_from_confusion(cm)
        h = g.history()
        row = {"backend": a.backend, "dtype": a.dtype, "clients": a.clients, "mu": mu, "rounds": int(h["rounds_run"]),
               "shard_sizes": [int(e.n_local) for e in g.clients],
               "train_global_round50": [float(x) for x in h["global"][-1]],
               "heldout": {k: float(v) for k, v in test.items()}, "wall_s": dt}
        res.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
