"""Entrypoint [H]: federated hyperparameter sweep (fedmi, packed trials).

Same grid, estimator settings and reporting as the reference ``hyperparameters_tuning.py``
(H:68-132): hidden_layer_sizes in 10 configs x learning_rate_init in 9 values,
MLPClassifier(relu, max_iter=400, random_state=42) per trial on the local contiguous shard,
uniform FedAvg of the weights, pooled global metrics, best trial by global accuracy.
Defaults to ``balanced_income_data.csv`` / ``income`` with ``StandardScaler(with_mean=False)``
(the reference names a diabetes CSV that is not shipped).

On a GPU the 9 learning rates of each hidden config train as one packed job
(``fedmi.hpo.sweep``).  ``--hidden`` / ``--lrs`` narrow the grid.

``--federated`` switches to the round-engine sweep of BASELINE config 5 (``fedmi.hpo.fed_sweep``):
a {hidden} x {lr} x {local steps per round} grid of multi-round FedAvg trials of the [C]
workload, ``--trials-per-gpu`` of them running concurrently on every GPU and sharing one
all-reduce per round.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 hyperparameters_tuning.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 hyperparameters_tuning.py --federated --rounds 50
"""
from __future__ import annotations

import argparse
import ast
import json
import sys
import time

import numpy as np

from fedmi.data.sharding import split_data
from fedmi.data.tabular import DEFAULT_DATASET, DEFAULT_LABEL, encode_categorical_features  # noqa: F401
from fedmi.data.tabular import load_tabular
from fedmi.fl.metrics import confusion_matrix, metrics_from_confusion
from fedmi.fl.sklearn_fed import average_estimator_weights
from fedmi.hpo.sweep import HIDDEN_GRID, LR_GRID, run_sweep
from fedmi.parallel.comm import get_world


class FederatedMLPLearning:
    """Reference [H] client API (hyperparameters_tuning.py:10-132) over fedmi components:
    ``_split_data`` (contiguous shard, H:17-22), ``federated_averaging`` (uniform mean of
    ``coefs_ + intercepts_``, H:24-46), ``_set_weights`` (H:48-54), ``_compute_metrics``
    (H:56-66) and ``train_and_evaluate`` -- the 10 x 9 grid of H:68-132, whose 9 learning
    rates per hidden config train as ONE packed job on the GPU (``fedmi.hpo.sweep``).
    ``train_and_evaluate`` returns ``(best_params, best_metrics, best_weights)`` like the
    reference's root rank prints them (H:126-132)."""

    def __init__(self, X, y, rank, size, comm=None, backend="auto", packed=True):
        self.rank = rank
        self.size = size
        self.comm = comm
        self.X_local, self.y_local = self._split_data(X, y, rank, size)
        self.local_model = None
        self.backend, self.packed = backend, packed

    def _split_data(self, X, y, rank, size):
        return split_data(X, y, rank, size, mode="contiguous")

    def federated_averaging(self, comm):
        global_weights = average_estimator_weights(self.local_model, comm, weighting="uniform")
        self._set_weights(global_weights)
        return global_weights

    def _set_weights(self, global_weights):
        k = len(self.local_model.coefs_)
        self.local_model.coefs_ = [np.array(w, dtype=np.float64) for w in global_weights[:k]]
        self.local_model.intercepts_ = [np.array(w, dtype=np.float64) for w in global_weights[k:]]

    def _compute_metrics(self, y_true, y_pred):
        return metrics_from_confusion(confusion_matrix(y_true, y_pred, 2))

    def train_and_evaluate(self, comm, rounds=1, hidden_grid=HIDDEN_GRID, lr_grid=LR_GRID, max_iter=400,
                           on_trial=None):
        best, results = None, []
        for _ in range(rounds):
            best, results = run_sweep(self.X_local, self.y_local, comm, hidden_grid, lr_grid, max_iter=max_iter,
                                      backend=self.backend, packed=self.packed, on_trial=on_trial)
        self.results = results
        if best is None:
            return None, None, None
        return ({"hidden_layer_sizes": best.hidden, "learning_rate": best.lr}, best.global_, best.weights)


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
    ap.add_argument("--save", default=None,
                    help="checkpoint directory (rank 0): trial results + every trial's averaged weights and the "
                         "best one as best.safetensors, coefs_ + intercepts_ layout (float64, [in, out])")
    ap.add_argument("--resume", default=None, help="reuse the trials of a sweep saved with --save")
    ap.add_argument("--federated", action="store_true",
                    help="round-engine sweep over hidden x lr x local steps (BASELINE config 5)")
    ap.add_argument("--local-steps", "--local-epochs", dest="local_steps", type=int, nargs="+", default=None,
                    help="--federated: local steps grid (one full-batch step = one local epoch)")
    ap.add_argument("--hpo-grid", default=None,
                    help='the whole grid as JSON, e.g. \'{"hidden": [[50, 200], [100]], "lr": [0.002, 0.004], '
                         '"local_steps": [1, 2]}\' (keys optional; overrides --hidden / --lrs / --local-steps)')
    ap.add_argument("--trials-per-gpu", type=int, default=6, help="--federated: concurrent trials per GPU")
    ap.add_argument("--dtype", choices=["fp64", "fp32", "bf16"], default=None,
                    help="sklearn sweep: estimator precision fp64 (default, sklearn's float64) | fp32; "
                         "--federated: engine MFMA dtype fp32 (default) | bf16")
    a = ap.parse_args(argv)
    if a.hpo_grid:
        grid_spec = json.loads(a.hpo_grid)
        unknown = set(grid_spec) - {"hidden", "lr", "local_steps"}
        if unknown:
            ap.error(f"--hpo-grid: unknown keys {sorted(unknown)}")
        if "hidden" in grid_spec:
            a.hidden = repr([tuple(int(x) for x in (h if isinstance(h, (list, tuple)) else [h]))
                             for h in grid_spec["hidden"]])
        if "lr" in grid_spec:
            a.lrs = [float(x) for x in grid_spec["lr"]]
        if "local_steps" in grid_spec:
            a.local_steps = [int(x) for x in grid_spec["local_steps"]]
    if a.federated:
        if a.dtype == "fp64":
            ap.error("--federated engines run fp32 or bf16")
        a.dtype = a.dtype or "fp32"
        return federated_main(a)
    if a.dtype == "bf16":
        ap.error("the sklearn sweep trains in fp64 or fp32")
    a.dtype = a.dtype or "fp64"
    comm = get_world(backend="gloo" if a.device == "cpu" else "auto", device=a.device)
    rank = comm.Get_rank()
    ds = load_tabular(a.data, label=a.label, with_mean=False)
    X_local, y_local = split_data(ds.X_train, ds.y_train, rank, comm.Get_size(), mode="contiguous")
    hidden = ast.literal_eval(a.hidden) if a.hidden else HIDDEN_GRID
    lrs = tuple(a.lrs) if a.lrs else LR_GRID
    backend = a.backend
    if backend == "auto":
        backend = "hip" if comm.device.type == "cuda" else "numpy"

    from fedmi.hpo.sweep import load_sweep, save_sweep
    from fedmi.parallel.consistency import digest
    # the run settings a checkpoint must match to be resumed (trials of another run, data or
    # client count must not mix into this run's best-trial selection)
    meta = {"world": comm.Get_size(), "max_iter": a.max_iter, "dtype": a.dtype,
            "data": digest([ds.X_train, ds.y_train])}
    done = load_sweep(a.resume, expect=meta) if a.resume else []
    partial = list(done)

    def report(res):
        partial.append(res)
        if a.save and rank == 0:
            save_sweep(a.save, partial, None, meta)  # incremental: a crash leaves a resumable sweep
        if a.quiet:
            return
        print("\n\tLOCAL MEASURED RESULTS\n")
        print(f"\t[Rank {rank}] Local Metrics (Hidden Layers: {res.hidden}, LR: {res.lr}): {res.local}\n", flush=True)
        print("-" * 50)
        if rank == 0:
            print("\nGLOBAL MEASURED RESULTS")
            print(f"\t[Rank {rank}] Global Metrics (Hidden Layers: {res.hidden}, LR: {res.lr}): {res.global_}\n")
            print("-" * 50, flush=True)

    if done and rank == 0:
        print(f"Resumed {len(done)} trials from {a.resume}", flush=True)
    t0 = time.time()
    best, results = None, []
    for rnd in range(a.rounds):
        if rank == 0:
            print(f"Training Round {rnd + 1}...\n{'-' * 50}")
        best, results = run_sweep(X_local, y_local, comm, hidden, lrs, max_iter=a.max_iter, backend=backend,
                                  packed=not a.no_pack, on_trial=report, done=done, dtype=a.dtype)
    wall = time.time() - t0
    if a.save and rank == 0:
        save_sweep(a.save, results, best, meta)
    comm.Barrier()
    if comm.Get_size() > 1:
        from fedmi.parallel.consistency import check_replicas
        check_replicas(comm, [np.asarray(w) for r in results for w in r.weights])  # every trial's average
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


def federated_main(a):
    """BASELINE config 5: federated {hidden, lr, local steps} sweep with packed trials."""
    from fedmi.fl.engine import EngineConfig
    from fedmi.hpo.fed_sweep import DEFAULT_HIDDEN, DEFAULT_LOCAL_STEPS, DEFAULT_LRS, grid, run_fed_sweep
    comm = get_world(backend="gloo" if a.device == "cpu" else "auto", device=a.device)
    rank, size = comm.Get_rank(), comm.Get_size()
    ds = load_tabular(a.data, label=a.label, with_mean=True)
    X_local, y_local = split_data(ds.X_train, ds.y_train, rank, size, mode="iid", seed=0)
    hidden = ast.literal_eval(a.hidden) if a.hidden else DEFAULT_HIDDEN
    trials = grid(hidden, tuple(a.lrs) if a.lrs else DEFAULT_LRS,
                  tuple(a.local_steps) if a.local_steps else DEFAULT_LOCAL_STEPS)
    rounds = a.rounds if a.rounds > 1 else 50
    # rows_per_block -1: trial batches take 64 rows per workgroup where LDS allows (bf16): half the
    # workgroups, and a packed group round is bound by workgroup slots x workgroup latency
    base = EngineConfig(max_rounds=rounds, dtype=a.dtype, graph_rounds=0, rows_per_block=-1)
    t0 = time.time()
    best, done = run_fed_sweep(X_local, y_local, 2, comm, trials, rounds=rounds, trials_per_gpu=a.trials_per_gpu,
                               base=base, backend="torch" if a.device == "cpu" else "auto")
    wall = time.time() - t0
    if size > 1:
        from fedmi.parallel.consistency import check_replicas
        check_replicas(comm, [np.asarray(t.history["global"]) for t in done])
    if rank == 0:
        for t in done:
            if not a.quiet:
                print(f"Trial hidden={t.hidden} lr={t.lr} local_steps={t.local_steps}: rounds={t.rounds_run} "
                      + ", ".join(f"{k}: {v:.4f}" for k, v in t.final.items()), flush=True)
        print(f"\nBest Global Hyperparameters: hidden={best.hidden} lr={best.lr} local_steps={best.local_steps}")
        print(f"Best Global Metrics: {best.final}")
        print(f"\nfederated sweep wall time: {wall:.2f} s for {len(done)} trials x {rounds} rounds "
              f"({a.trials_per_gpu} concurrent per GPU, {size} clients)", flush=True)
        if a.json:
            with open(a.json, "w") as f:
                json.dump([{"hidden": t.hidden, "lr": t.lr, "local_steps": t.local_steps, "rounds": t.rounds_run,
                            "final": t.final} for t in done] + [{"wall_s": wall}], f)
    comm.close()
    return best, done


if __name__ == "__main__":
    main(sys.argv[1:])
