"""Entrypoint [H]: federated hyperparameter sweep (fedmi, packed trials).

Same grid, estimator settings and reporting as the reference ``hyperparameters_tuning.py``
(H:68-132): hidden_layer_sizes in 10 configs x learning_rate_init in 9 values,
MLPClassifier(relu, max_iter=400, random_state=42) per trial on the local contiguous shard,
uniform FedAvg of the weights, pooled global metrics, best trial by global accuracy.
Defaults to ``balanced_income_data.csv`` / ``income`` with ``StandardScaler(with_mean=False)``
(the reference names a diabetes CSV that is not shipped).

On a GPU the 9 learning rates of each hidden config train as one packed job
(``fedmi.hpo.sweep``).  ``--hidden`` / ``--lrs`` narrow the grid.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 hyperparameters_tuning.py
"""
from __future__ import annotations

import argparse
import ast
import json
import sys
import time

import numpy as np

from fedmi.data.sharding import split_data
from fedmi.data.tabular import DEFAULT_DATASET, DEFAULT_LABEL, load_tabular
from fedmi.hpo.sweep import HIDDEN_GRID, LR_GRID, run_sweep
from fedmi.parallel.comm import get_world


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data", default=DEFAULT_DATASET)
    ap.add_argument("--label", default=DEFAULT_LABEL)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--hidden", default=None, help="python literal list of tuples, e.g. '[(50,), (50, 200)]'")
    ap.add_argument("--lrs", type=float, nargs="+", default=None)
    ap.add_argument("--max-iter", type=int, default=400)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--backend", default="auto", help="estimator backend: hip | numpy")
    ap.add_argument("--no-pack", action="store_true", help="fit trials one by one")
    ap.add_argument("--quiet", action="store_true", help="only print the best result")
    ap.add_argument("--json", default=None, help="write all trial results here (rank 0)")
    a = ap.parse_args(argv)
    comm = get_world(backend="gloo" if a.device == "cpu" else "auto", device=a.device)
    rank = comm.Get_rank()
    ds = load_tabular(a.data, label=a.label, with_mean=False)
    X_local, y_local = split_data(ds.X_train, ds.y_train, rank, comm.Get_size(), mode="contiguous")
    hidden = ast.literal_eval(a.hidden) if a.hidden else HIDDEN_GRID
    lrs = tuple(a.lrs) if a.lrs else LR_GRID
    backend = a.backend
    if backend == "auto":
        backend = "hip" if comm.device.type == "cuda" else "numpy"

    def report(res):
        if a.quiet:
            return
        print("\n\tLOCAL MEASURED RESULTS\n")
        print(f"\t[Rank {rank}] Local Metrics (Hidden Layers: {res.hidden}, LR: {res.lr}): {res.local}\n", flush=True)
        print("-" * 50)
        if rank == 0:
            print("\nGLOBAL MEASURED RESULTS")
            print(f"\t[Rank {rank}] Global Metrics (Hidden Layers: {res.hidden}, LR: {res.lr}): {res.global_}\n")
            print("-" * 50, flush=True)

    t0 = time.time()
    best, results = None, []
    for rnd in range(a.rounds):
        if rank == 0:
            print(f"Training Round {rnd + 1}...\n{'-' * 50}")
        best, results = run_sweep(X_local, y_local, comm, hidden, lrs, max_iter=a.max_iter, backend=backend,
                                  packed=not a.no_pack, on_trial=report)
    wall = time.time() - t0
    if rank == 0:
        print("\n\nBest MEASURED RESULTS")
        print("\nBest Global Hyperparameters:", {"hidden_layer_sizes": best.hidden, "learning_rate": best.lr})
        print(f"Best Global Metrics: {best.global_}")
        if not a.quiet:
            print("\nBest Global Weights:")
            for idx, w in enumerate(best.weights):
                print(f"Layer {idx + 1}: {w.shape}\n{w}")
        print(f"\nsweep wall time: {wall:.2f} s for {len(results)} trials", flush=True)
        if a.json:
            with open(a.json, "w") as f:
                json.dump([{"hidden": r.hidden, "lr": r.lr, "local": r.local, "global": r.global_,
                            "n_iter": r.n_iter} for r in results] + [{"wall_s": wall}], f)
    comm.close()
    return best, results


if __name__ == "__main__":
    main(sys.argv[1:])
