"""Federated averaging helpers for scikit-learn-style estimators ([S]/[H] flows).

Reference: root-centric ``gather(coefs_ + intercepts_)`` -> ``np.mean`` per layer ->
``bcast`` (``FL_SkLearn_MLPClassifier_Limitation.py:108-122``,
``hyperparameters_tuning.py:24-46``) and ``gather(y_true)`` / ``gather(y_pred)`` for pooled
metrics (S:126-134).  Here: one in-place SUM all-reduce of the flattened parameter list
(uniform mean, SURVEY Q9, or sample-size weighted) and one all-reduce of the C x C
confusion matrix (pooled metrics are a function of it, Q4).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch


def _allreduce_np(x: np.ndarray, comm) -> np.ndarray:
    if comm is None or comm.size == 1:
        return x
    t = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64))
    if comm.device.type == "cuda" and comm.backend != "gloo":
        t = t.to(comm.device)
        comm.allreduce_(t)
        return t.cpu().numpy()
    import torch.distributed as dist
    dist.all_reduce(t)
    return t.numpy()


def average_estimator_weights(est, comm, weighting: str = "uniform", n_local: int = 0) -> List[np.ndarray]:
    """Average ``coefs_ + intercepts_`` over ranks; returns the global list (same shapes)."""
    arrs = list(est.coefs_) + list(est.intercepts_)
    flat = np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in arrs])
    size = 1 if comm is None else comm.size
    if weighting == "uniform":
        flat = _allreduce_np(flat / size, comm)
    else:
        tot = _allreduce_np(np.array([float(n_local)]), comm)[0]
        flat = _allreduce_np(flat * (n_local / tot), comm)
    out, off = [], 0
    for a in arrs:
        n = np.asarray(a).size
        out.append(flat[off:off + n].reshape(np.asarray(a).shape))
        off += n
    return out


def allreduce_confusion(cm: np.ndarray, comm) -> np.ndarray:
    return _allreduce_np(cm.astype(np.float64), comm).round().astype(np.int64)


def average_many_estimator_weights(ests, comm) -> List[List[np.ndarray]]:
    """:func:`average_estimator_weights` (uniform) of several estimators in ONE all-reduce: every
    estimator's flattened ``coefs_ + intercepts_`` / size side by side.  Each element gets the same
    arithmetic as its own all-reduce (divided by the size, then summed over the ranks; the order of
    that sum is the backend's -- gloo's and RCCL's depend on the buffer's length, the device host
    plane's is rank order); the [H] sweep averages its 90 trials this way instead of with 90
    all-reduces."""
    size = 1 if comm is None else comm.size
    layouts, flats = [], []
    for est in ests:
        arrs = list(est.coefs_) + list(est.intercepts_)
        layouts.append([np.asarray(a).shape for a in arrs])
        flats.append(np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in arrs]))
    if not flats:
        return []
    flat = _allreduce_np(np.concatenate(flats) / size, comm)
    out, off = [], 0
    for shapes in layouts:
        ws = []
        for shp in shapes:
            n = int(np.prod(shp))
            ws.append(flat[off:off + n].reshape(shp))
            off += n
        out.append(ws)
    return out

