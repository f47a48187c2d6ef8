"""Federated hyperparameter sweep with trial packing (reference [H]).

Reference ``hyperparameters_tuning.py:68-132`` runs 10 hidden-layer configs x 9 learning
rates = 90 trials *sequentially*; for each: fit a fresh ``MLPClassifier(hl, lr,
max_iter=400, random_state=42)`` on the local shard, local metrics, uniform FedAvg of the
weights, pooled global metrics (of the *local* predictions), and keep the best trial by
global accuracy together with its averaged weights.

Here the 9 learning rates of one hidden config are one packed device job
(:func:`fedmi.models.sklearn_mlp.fit_packed`): same architecture, same random_state ->
same initial weights and minibatch permutations, so every minibatch is gathered once and
fed to 9 models through batched MFMA GEMMs, with per-trial learning rate, loss and
early-stop state on the device.  Results are identical in semantics to 9 separate fits.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..fl.metrics import confusion_matrix, metrics_from_confusion
from ..fl.sklearn_fed import allreduce_confusion, average_many_estimator_weights
from ..models.sklearn_mlp import MLPClassifier, fit_packed, packed_inputs, prepare_packed

HIDDEN_GRID: Tuple[Tuple[int, ...], ...] = ((50,), (100,), (50, 50), (100, 50), (50, 100), (50, 200), (50, 400),
                                            (100, 400), (400, 200), (200, 400))
LR_GRID: Tuple[float, ...] = (0.002, 0.005, 0.004, 0.008, 0.01, 0.02, 0.05, 0.1, 0.2)


@dataclass
class TrialResult:
    hidden: Tuple[int, ...]
    lr: float
    local: Dict[str, float]
    global_: Dict[str, float]
    n_iter: int
    weights: List[np.ndarray] = field(repr=False, default_factory=list)


def run_sweep(X_local, y_local, comm, hidden_grid: Sequence = HIDDEN_GRID, lr_grid: Sequence = LR_GRID,
              max_iter: int = 400, random_state: int = 42, backend: str = "auto", packed: bool = True,
              on_trial=None, done: Sequence[TrialResult] = (),
              dtype: str = "float64") -> Tuple[Optional[TrialResult], List[TrialResult]]:
    """``done``: results of an earlier (checkpointed) sweep; their hidden configs are not trained
    again and the best trial is taken over old and new results in grid order."""
    classes = np.unique(y_local)
    n_cls = max(2, len(classes))
    have = {(tuple(r.hidden), float(r.lr)): r for r in done}
    todo = [hl for hl in hidden_grid if any((tuple(hl), float(lr)) not in have for lr in lr_grid)]
    fresh = _train(X_local, y_local, comm, todo, lr_grid, max_iter, random_state, backend, packed, n_cls, on_trial,
                   dtype)
    results = [have.get((tuple(hl), float(lr))) or fresh[(tuple(hl), float(lr))] for hl in hidden_grid
               for lr in lr_grid]
    best: Optional[TrialResult] = None
    for res in results:
        if best is None or res.global_["accuracy"] > best.global_["accuracy"]:
            best = res
    return best, results


def _predict_device(ests: Sequence[MLPClassifier], X) -> List[np.ndarray]:
    """``[e.predict(X) for e in ests]`` as float64 products on the GPU (the host's numpy forward
    took 0.74 s of the 3.4 s reference sweep: 8000 x 200 x 400 products for 90 trials,
    profiles/h_sweep_phases_r6.log).  The same formula as MLPClassifier.predict -- ReLU hidden
    layers, logistic > 0.5 or softmax argmax -- so only a row whose output sits within rounding of
    the decision boundary could come out differently (tests/test_sklearn_estimator.py pins the
    sweep's metrics to the host forward)."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float64), device=dev)
    out = []
    for e in ests:
        a = x
        L = len(e.coefs_)
        for i, (W, b) in enumerate(zip(e.coefs_, e.intercepts_)):
            a = torch.addmm(torch.as_tensor(b, device=dev), a, torch.as_tensor(W, device=dev))
            if i < L - 1:
                a = torch.relu(a)
        idx = (torch.sigmoid(a.ravel()) > 0.5).long() if e.n_outputs_ == 1 else torch.argmax(a, dim=1)
        out.append(e.classes_[idx.cpu().numpy()])
    return out


def _train(X_local, y_local, comm, hidden_grid, lr_grid, max_iter, random_state, backend, packed, n_cls, on_trial,
           dtype="float64"):
    import os
    import sys
    import time
    timing = os.environ.get("FEDMI_SWEEP_TIMING", "0") == "1"   # phase times on stderr
    t_start = time.perf_counter()
    out = {}
    groups = [[MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=lr, max_iter=max_iter,
                             random_state=random_state, backend=backend, dtype=dtype) for lr in lr_grid]
              for hl in hidden_grid]
    # Training needs no communication (every trial fits from scratch, Q8): on the GPU the
    # packed jobs of all hidden configs run concurrently, one host thread + stream each (the
    # native epoch loop releases the GIL; each job's kernels are far too small to fill the
    # GPU alone).  Averaging and pooled metrics then follow in the reference's trial order,
    # so every rank issues its collectives in the same sequence.
    if packed and groups and groups[0][0]._resolve_backend() == "hip" and len(groups) > 1:
        from concurrent.futures import ThreadPoolExecutor
        # every job is built and its epoch graph captured HERE, one after another, before any
        # thread starts: a capture overlapping another thread's allocations / copies / polling
        # was invalidated (ranks sharing a GPU made the overlap likely); the threads then only
        # replay graphs and poll, and the results are copied back here
        # the host halves (estimator init + epoch orders, GIL-free in the native generator) of every
        # job concurrently; then the device halves one after another
        # (only with integer random_states: a shared RandomState must not be drawn from two threads)
        own_rng = all(isinstance(g[0].random_state, (int, np.integer)) for g in groups)
        with ThreadPoolExecutor(max_workers=min(8, len(groups)) if own_rng else 1) as ex:
            inputs = list(ex.map(lambda g: packed_inputs(g, X_local, y_local), groups))
        jobs = [prepare_packed(ests, X_local, y_local, inputs=inp) for ests, inp in zip(groups, inputs)]
        t_prep = time.perf_counter()

        def run_timed(j):
            t0 = time.perf_counter()
            j.run()
            return time.perf_counter() - t0

        # FEDMI_SWEEP_RUN_THREADS=1 replays the jobs one after another (profiling: rocprofv3's kernel trace
        # crashed inside hipGraphLaunch with ten threads replaying graphs, profiles/h_sweep_kernels_r6.txt)
        n_run = int(os.environ.get("FEDMI_SWEEP_RUN_THREADS", "0") or 0) or len(jobs)
        with ThreadPoolExecutor(max_workers=min(n_run, len(jobs))) as ex:
            job_s = list(ex.map(run_timed, jobs))
        t_run = time.perf_counter()
        for j in jobs:
            j.finish()
        if timing:
            print(f"[sweep] prepare (build + capture) {t_prep - t_start:.3f} s, concurrent runs {t_run - t_prep:.3f} s, "
                  f"finish {time.perf_counter() - t_run:.3f} s; per job: "
                  + ", ".join(f"{tuple(g[0].hidden_layer_sizes)} {t:.3f} s" for g, t in zip(groups, job_s)),
                  file=sys.stderr, flush=True)
    elif packed:
        for ests in groups:
            fit_packed(ests, X_local, y_local)
    else:
        for ests in groups:
            for e in ests:
                e.fit(X_local, y_local)
    on_device = packed and bool(groups) and groups[0][0]._resolve_backend() == "hip"
    trials, cms = [], []
    for hl, ests in zip(hidden_grid, groups):
        preds = _predict_device(ests, X_local) if on_device else [e.predict(X_local) for e in ests]
        for lr, est, y_pred in zip(lr_grid, ests, preds):
            trials.append((hl, lr, est))
            cms.append(confusion_matrix(y_local, y_pred, n_cls))
    # every trial's FedAvg (uniform mean of coefs_ + intercepts_, H:24-46) and pooled confusion in
    # TWO all-reduces instead of two per trial -- the same per-element arithmetic
    gws = average_many_estimator_weights([est for _, _, est in trials], comm)
    pooled = allreduce_confusion(np.stack(cms), comm) if cms else []
    for (hl, lr, est), cm_local, gw, cm in zip(trials, cms, gws, pooled):
        k = len(est.coefs_)
        est.coefs_, est.intercepts_ = gw[:k], gw[k:]
        res = TrialResult(tuple(hl), float(lr), metrics_from_confusion(cm_local), metrics_from_confusion(cm),
                          int(est.n_iter_), [np.copy(w) for w in gw])
        out[(tuple(hl), float(lr))] = res
        if on_trial is not None:
            on_trial(res)
    if timing:
        print(f"[sweep] total {time.perf_counter() - t_start:.3f} s (metrics + FedAvg of every trial included)",
              file=sys.stderr, flush=True)
    return out


def _trial_file(r: TrialResult) -> str:
    # repr(lr): the shortest string that round-trips the float, so nearby grid rates never share a file
    return "trial_h" + "-".join(str(h) for h in r.hidden) + f"_lr{float(r.lr)!r}.safetensors"


def _trial_tag(r: TrialResult) -> str:
    return "-".join(str(h) for h in r.hidden) + "|" + repr(float(r.lr))


def _run_key(meta: dict) -> str:
    """The run settings a trial file belongs to (sweep.json's metadata, without the trial list)."""
    import json
    return json.dumps({k: v for k, v in meta.items() if k not in ("trials", "best")}, sort_keys=True, default=str)


def save_sweep(path: str, results: Sequence[TrialResult], best: Optional[TrialResult], meta: dict) -> None:
    """[H] checkpoint: every trial's metrics (JSON) + the best trial's averaged weights in the
    reference's coefs_ + intercepts_ layout (H:119, H:130-132) as ``best.safetensors``.
    Incremental: called after every finished trial (hyperparameters_tuning.py).  A trial's weights
    file is skipped only when the directory's current ``sweep.json`` is of THIS run (same metadata)
    and already lists that file; anything else is (re)written to a temporary name and renamed, so a
    directory left by another run never lends its weights to this one.  Every file's
    header names its trial and run, checked by :func:`load_sweep`; ``sweep.json`` is replaced last,
    atomically, so a crash part-way leaves a resumable sweep of the trials done."""
    import json
    import os
    from ..ckpt.checkpoint import _publish_meta
    from safetensors.numpy import save_file
    os.makedirs(path, exist_ok=True)
    # one result per (hidden, lr), the latest: a resumed, partly-done hidden config retrains some
    # rates that `done` already holds
    uniq = {}
    for r in results:
        uniq[(tuple(r.hidden), float(r.lr))] = r
    results = list(uniq.values())
    key = _run_key(meta)
    trusted = set()
    sj = os.path.join(path, "sweep.json")
    if os.path.isfile(sj):
        try:
            with open(sj) as f:
                old = json.load(f)
            if _run_key(old) == key:
                trusted = {t.get("file") for t in old.get("trials", [])}
        except (OSError, ValueError):
            trusted = set()

    def write(fp, w, tag):
        ws = [np.ascontiguousarray(np.asarray(x, dtype=np.float64)) for x in w]
        L = len(ws) // 2
        t = {f"coefs_.{i}": ws[i] for i in range(L)}
        t.update({f"intercepts_.{i}": ws[L + i] for i in range(L)})
        tmp = fp + f".tmp{os.getpid()}"
        save_file(t, tmp, metadata={"trial": tag, "run": key})
        os.replace(tmp, fp)

    for r in results:
        name = _trial_file(r)
        fp = os.path.join(path, name)
        if name not in trusted or not os.path.isfile(fp):
            write(fp, r.weights, _trial_tag(r))
    if best is not None:
        write(os.path.join(path, "best.safetensors"), best.weights, _trial_tag(best))
    rows = [{"hidden": list(r.hidden), "lr": r.lr, "local": r.local, "global": r.global_, "n_iter": r.n_iter,
             "file": _trial_file(r)} for r in results]
    _publish_meta(path, dict(meta, trials=rows, best={"hidden": list(best.hidden), "lr": best.lr} if best else None),
                  name="sweep.json")


def load_sweep(path: str, expect: Optional[dict] = None) -> List[TrialResult]:
    """Trials of a saved sweep.  ``expect``: run settings (world, max_iter, data digest, ...)
    that must equal the saved ones -- trials of a different run must not mix into this one's
    best-trial selection.  Each weights file must carry its trial's and this run's tag."""
    import json
    import os
    from safetensors import safe_open
    from ..ckpt.checkpoint import load_sklearn_weights
    with open(os.path.join(path, "sweep.json")) as f:
        m = json.load(f)
    for k, v in (expect or {}).items():
        if m.get(k) != v:
            raise ValueError(f"{path}: saved with {k}={m.get(k)!r}, this run has {k}={v!r}; not resuming")
    key = _run_key(m)
    out = []
    for i, r in enumerate(m["trials"]):
        fp = os.path.join(path, r.get("file", f"trial{i}.safetensors"))
        res = TrialResult(tuple(r["hidden"]), float(r["lr"]), r["local"], r["global"], int(r["n_iter"]), [])
        with safe_open(fp, framework="numpy") as f:
            md = f.metadata() or {}
        if "trial" in md and (md["trial"] != _trial_tag(res) or md.get("run") != key):
            raise ValueError(f"{fp}: weights of trial {md['trial']!r} of another run, not of {_trial_tag(res)!r}")
        res.weights = load_sklearn_weights(fp)
        out.append(res)
    return out
