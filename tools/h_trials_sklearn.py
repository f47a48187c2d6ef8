"""Fit the [H] grid (hyperparameters_tuning.py:83-112, k clients) with scikit-learn on the CPU, one trial per worker.

Writes one JSON row per trial (hidden, lr, pooled training accuracy, n_iter_) so the HIP sweep's per-trial values
(`hyperparameters_tuning.py --save`) can be compared with tools/h_trials_compare.py.  Workers run with one BLAS
thread each (the BASELINE.md set-up) unless --blas-threads says otherwise.

    python tools/h_trials_sklearn.py --out profiles/h_trials_sklearn_1thr.json --workers 8
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _fit(args):
    hidden, lr, max_iter, clients = args
    import warnings
    import numpy as np
    from sklearn.neural_network import MLPClassifier
    from fedmi.data.sharding import split_data
    from fedmi.data.tabular import load_tabular
    warnings.filterwarnings("ignore")
    ds = load_tabular(with_mean=False)
    t = time.perf_counter()
    hits, n_iter = 0, []
    for r in range(clients):   # each client's local fit and local predictions, pooled (H:91-112)
        X, y = split_data(ds.X_train, ds.y_train, r, clients, mode="contiguous")
        c = MLPClassifier(activation="relu", hidden_layer_sizes=hidden, learning_rate_init=lr, max_iter=max_iter,
                          random_state=42).fit(X, y)
        hits += int(np.sum(c.predict(X) == y))
        n_iter.append(int(c.n_iter_))
    acc = hits / len(ds.y_train)
    return {"hidden": list(hidden), "lr": lr, "accuracy": acc, "n_iter": n_iter[0], "n_iter_clients": n_iter,
            "fit_s": round(time.perf_counter() - t, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--blas-threads", type=int, default=1)
    ap.add_argument("--max-iter", type=int, default=400)
    ap.add_argument("--clients", type=int, default=1, help="k contiguous shards (hyperparameters_tuning.py:17-22)")
    a = ap.parse_args()
    for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[k] = str(a.blas_threads)   # set before the workers import numpy
    from fedmi.hpo.sweep import HIDDEN_GRID, LR_GRID
    jobs = [(h, lr, a.max_iter, a.clients) for h in HIDDEN_GRID for lr in LR_GRID]
    jobs.sort(key=lambda j: -sum(j[0]))        # the long fits first
    with ProcessPoolExecutor(a.workers) as ex:
        rows = list(ex.map(_fit, jobs))
    with open(a.out, "w") as f:
        json.dump({"blas_threads": a.blas_threads, "max_iter": a.max_iter, "clients": a.clients, "trials": rows}, f, indent=1)
    print(f"{len(rows)} trials -> {a.out}")


if __name__ == "__main__":
    main()
