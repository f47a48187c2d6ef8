"""Classification metrics from a confusion matrix.

The reference computes accuracy and *weighted* precision / recall / F1 with
``zero_division=0`` through sklearn on host arrays of predictions
(``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:85-90``,
``FL_SkLearn_MLPClassifier_Limitation.py:56-66``).  All four are functions of the C x C
confusion matrix, which is what the device produces (``argmax_confusion`` /
``eval_confusion`` kernels) and what crosses the network: a few integers per client
instead of the reference's gathered ``y_true``/``y_pred`` vectors (S:126-134).

``metrics_from_confusion`` matches sklearn to fp64 rounding; ``pooled`` (micro) vs
``mean_over_clients`` reproduce the two "global metric" conventions of the reference
(SURVEY Q3 for [C], Q4 for [S]/[H]).
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

METRIC_NAMES = ("accuracy", "precision", "recall", "f1")


def confusion_matrix(y_true: np.ndarray, y_pred: np.ndarray, n_classes: int) -> np.ndarray:
    cm = np.zeros((n_classes, n_classes), dtype=np.int64)
    np.add.at(cm, (np.asarray(y_true, dtype=np.int64), np.asarray(y_pred, dtype=np.int64)), 1)
    return cm


def metrics_from_confusion(cm) -> Dict[str, float]:
    """cm[t][p] = count of rows with true class t predicted as p."""
    cm = np.asarray(cm, dtype=np.float64)
    total = cm.sum()
    if total == 0:
        return {k: 0.0 for k in METRIC_NAMES}
    tp = np.diag(cm)
    support = cm.sum(axis=1)
    predicted = cm.sum(axis=0)
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(predicted > 0, tp / predicted, 0.0)
        rec = np.where(support > 0, tp / support, 0.0)
        denom = 2 * tp + (predicted - tp) + (support - tp)
        f1 = np.where(denom > 0, 2 * tp / denom, 0.0)
    w = support / support.sum()
    return {
        "accuracy": float(tp.sum() / total),
        "precision": float((w * prec).sum()),
        "recall": float((w * rec).sum()),
        "f1": float((w * f1).sum()),
    }


def metric_vector(m: Dict[str, float]) -> np.ndarray:
    return np.array([m[k] for k in METRIC_NAMES], dtype=np.float64)


def mean_over_clients(per_client: Sequence[Dict[str, float]]) -> Dict[str, float]:
    """[C] convention: unweighted mean of per-client metrics (C:169)."""
    return {k: float(np.mean([m[k] for m in per_client])) for k in METRIC_NAMES}


def pooled(cms: Sequence[np.ndarray]) -> Dict[str, float]:
    """[S]/[H] convention: metrics of the concatenated predictions (S:130-134, Q4)
    == metrics of the summed confusion matrices."""
    return metrics_from_confusion(np.sum(np.stack([np.asarray(c) for c in cms]), axis=0))


def format_metrics(m: Dict[str, float]) -> str:
    return (f"[accuracy: {m['accuracy']:.4f}, precision: {m['precision']:.4f}, "
            f"recall: {m['recall']:.4f}, f1: {m['f1']:.4f}]")
