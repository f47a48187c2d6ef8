"""Entrypoint [S]: federated averaging of scikit-learn-style MLPClassifiers (fedmi).

Same flow and defaults as the reference ``FL_SkLearn_MLPClassifier_Limitation.py``
(S:68-153): MLPClassifier((50, 400), relu, lr 0.004, max_iter 300, random_state 42),
``partial_fit`` to initialise, then per round: apply the global weights, ``fit`` on the
local contiguous shard, local metrics, uniform FedAvg of ``coefs_ + intercepts_``, pooled
global metrics; at the end per-layer mean/std of the global weights.  Data:
``balanced_income_data.csv`` / ``income`` with ``StandardScaler(with_mean=False)`` (S:184).

The estimator is fedmi's ``MLPClassifier``: on a GPU the native HIP minibatch trainer in
float64 by default (f64 MFMA, scikit-learn's numerics; ``--dtype float32`` for the fp32
kernels), on a CPU the float64 numpy backend.  The reference's limitation is kept by default (``fit`` re-initialises, so the
averaged weights are discarded: SURVEY Q8); ``--warm-start`` fixes it.  FedAvg is one
in-place all-reduce of the flat parameter vector (uniform mean, S:114-117), and
the pooled metrics come from all-reduced confusion matrices instead of gathered
``y_true``/``y_pred`` arrays (S:126-134).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 FL_SkLearn_MLPClassifier_Limitation.py
"""
from __future__ import annotations

import argparse
import sys

import numpy as np
import torch

from fedmi.data.sharding import split_data
from fedmi.data.tabular import DEFAULT_DATASET, DEFAULT_LABEL, load_tabular
from fedmi.fl.metrics import confusion_matrix, metrics_from_confusion
from fedmi.fl.sklearn_fed import allreduce_confusion, average_estimator_weights
from fedmi.models.sklearn_mlp import MLPClassifier
from fedmi.parallel.comm import get_world


class FederatedMLPLearning:
    """Reference [S] client API (S:10-66) over fedmi components."""

    def __init__(self, X, y, rank, size, comm=None, hidden=(50, 400), lr=0.004, max_iter=300, warm_start=False,
                 backend="auto", dtype="float64"):
        self.rank = rank
        self.size = size
        self.comm = comm
        self.X_local, self.y_local = self._split_data(X, y, rank, size)
        self.local_model = None
        self.global_weights = None
        self.hidden, self.lr, self.max_iter = hidden, lr, max_iter
        self.warm_start, self.backend, self.dtype = warm_start, backend, dtype

    def _split_data(self, X, y, rank, size):
        return split_data(X, y, rank, size, mode="contiguous")

    def _set_weights(self, global_weights):
        k = len(self.local_model.coefs_)
        self.local_model.coefs_ = [np.array(w, dtype=np.float64) for w in global_weights[:k]]
        self.local_model.intercepts_ = [np.array(w, dtype=np.float64) for w in global_weights[k:]]

    def _compute_metrics(self, y_true, y_pred):
        return metrics_from_confusion(confusion_matrix(y_true, y_pred, 2))

    def federated_averaging(self, comm):
        self.global_weights = average_estimator_weights(self.local_model, comm, weighting="uniform")
        self._set_weights(self.global_weights)

    def train_and_evaluate(self, comm, rounds=1, save=None, resume=None):
        """S:68-153.  ``save``: checkpoint directory written after every round in the reference's
        exchange layout (coefs_ + intercepts_, float64 [in, out]); ``resume``: continue such a run."""
        from fedmi.ckpt.checkpoint import load_sklearn_run, save_sklearn_run
        self.local_model = MLPClassifier(activation="relu", hidden_layer_sizes=self.hidden,
                                         learning_rate_init=self.lr, max_iter=self.max_iter, random_state=42,
                                         warm_start=self.warm_start, backend=self.backend, dtype=self.dtype)
        classes = np.unique(self.y_local)
        self.local_model.partial_fit(self.X_local, self.y_local, classes=classes)
        history = []
        start = 0
        if resume:
            ck = load_sklearn_run(resume, self.rank)
            m = ck["meta"]
            if list(m["hidden"]) != list(self.hidden) or int(m["world"]) != self.size:
                raise ValueError(f"{resume}: saved for hidden {m['hidden']} x {m['world']} clients")
            start, history = int(m["rounds"]), list(m["history"])
            self.global_weights = ck["global"]
            self._set_weights(ck["local"])
            if self.rank == 0:
                print(f"Resumed from {resume} after {start} rounds", flush=True)
        for rnd in range(start, rounds):
            print(f"\n[Rank {self.rank}] Starting Round {rnd + 1}", flush=True)
            if rnd > 0 and self.global_weights is not None:
                self._set_weights(self.global_weights)
                print(f"[Rank {self.rank}] Applied global weights at the start of Round {rnd + 1}", flush=True)
            self.local_model.fit(self.X_local, self.y_local)
            y_pred = self.local_model.predict(self.X_local)
            local_metrics = self._compute_metrics(self.y_local, y_pred)
            print(f"[Rank {self.rank}] Local Metrics after training (Round {rnd + 1}): {local_metrics}", flush=True)
            self.global_weights = average_estimator_weights(self.local_model, comm, weighting="uniform")
            if self.rank == 0:
                print(f"[Rank {self.rank}] Computed global weights after Round {rnd + 1}", flush=True)
            cm = allreduce_confusion(confusion_matrix(self.y_local, y_pred, 2), comm)
            g = metrics_from_confusion(cm)
            history.append({"local": local_metrics, "global": g, "n_iter": int(self.local_model.n_iter_)})
            if self.rank == 0:
                print(f"\n[Rank {self.rank}] Global Metrics for Round {rnd + 1}:")
                print(f"  Accuracy: {g['accuracy']:.4f}")
                print(f"  Precision: {g['precision']:.4f}")
                print(f"  Recall: {g['recall']:.4f}")
                print(f"  F1: {g['f1']:.4f}")
                print("-" * 50, flush=True)
            if comm is not None:
                comm.Barrier()
            if save:
                save_sklearn_run(save, self.rank, rnd + 1, self.global_weights,
                                 list(self.local_model.coefs_) + list(self.local_model.intercepts_),
                                 {"hidden": list(self.hidden), "lr": self.lr, "max_iter": self.max_iter,
                                  "warm_start": self.warm_start, "world": self.size, "history": history}, comm)
        if comm is not None and comm.size > 1 and self.global_weights is not None:
            from fedmi.parallel.consistency import check_replicas
            check_replicas(comm, self.global_weights)  # every client holds the same average
        if self.rank == 0 and self.global_weights is not None:
            print("\nFinal Global Weight Statistics:")
            for idx, w in enumerate(self.global_weights):
                print(f"Layer {idx + 1} - Shape: {w.shape}")
                print(f"Mean: {np.mean(w):.6f}, Std: {np.std(w):.6f}", flush=True)
        return history


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data", default=DEFAULT_DATASET)
    ap.add_argument("--label", default=DEFAULT_LABEL)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--hidden", type=int, nargs="+", default=[50, 400])
    ap.add_argument("--lr", type=float, default=0.004)
    ap.add_argument("--max-iter", type=int, default=300)
    ap.add_argument("--warm-start", action="store_true", help="keep the averaged weights across rounds (fixes Q8)")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--backend", default="auto", help="estimator backend: hip | numpy")
    ap.add_argument("--dtype", default="float64", choices=["float64", "float32"],
                    help="HIP backend precision (float64 = sklearn's numerics, f64 MFMA)")
    ap.add_argument("--save", default=None, help="checkpoint directory (coefs_ + intercepts_ layout), every round")
    ap.add_argument("--resume", default=None, help="continue a run saved with --save")
    a = ap.parse_args(argv)
    comm = get_world(backend="gloo" if a.device == "cpu" else "auto", device=a.device)
    ds = load_tabular(a.data, label=a.label, with_mean=False)
    backend = a.backend
    if backend == "auto":
        backend = "hip" if comm.device.type == "cuda" else "numpy"
    tr = FederatedMLPLearning(ds.X_train, ds.y_train, comm.rank, comm.size, comm=comm, hidden=tuple(a.hidden),
                              lr=a.lr, max_iter=a.max_iter, warm_start=a.warm_start, backend=backend,
                              dtype=a.dtype)
    hist = tr.train_and_evaluate(comm, rounds=a.rounds, save=a.save, resume=a.resume)
    comm.close()
    return hist


if __name__ == "__main__":
    main(sys.argv[1:])
