"""One packed config-5 group (12 trials: hidden {(50,200),(100,50),(50,100)} x lr {0.002,0.004} x
local steps {1,2}) on one GPU, `--rows` rows per trial, `--rounds` graph-replayed rounds: the
region rocprofv3 traces for the per-kernel breakdown of a packed round
(tools/trace_by_grid.py).  Prints the trial-round time."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedmi.data.synthetic import make_income_like  # noqa: E402
from fedmi.fl.engine import EngineConfig  # noqa: E402
from fedmi.hpo.fed_sweep import FedTrialGroup, grid  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8000)
    ap.add_argument("--rounds", type=int, default=160)
    ap.add_argument("--same", action="store_true", help="one shape: (50, 200) x 6 lr x 2 local steps")
    a = ap.parse_args()
    X, y = make_income_like(a.rows, seed=1)
    trials = grid(((50, 200),), (0.001, 0.002, 0.003, 0.004, 0.006, 0.01), (1, 2)) if a.same else \
        grid(((50, 200), (100, 50), (50, 100)), (0.002, 0.004), (1, 2))
    base = EngineConfig(max_rounds=a.rounds + 48, early_stop=False, dtype="bf16", graph_rounds=16)
    g = FedTrialGroup(X, y, 2, trials, None, base)
    g.run(16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.run(a.rounds)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{len(trials)} trials x {a.rounds} rounds, {a.rows} rows: {dt / (a.rounds * len(trials)) * 1e6:.2f} us "
          f"per trial-round; batches {[(b.hidden if hasattr(b, 'hidden') else '?') for b in g.batches]}", flush=True)


if __name__ == "__main__":
    main()
