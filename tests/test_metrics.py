"""Device-metric formulas vs sklearn (C:85-90) and the early-stop oracle (C:181-192)."""
import numpy as np
import pytest

from fedmi.fl.early_stop import EarlyStopper, allclose
from fedmi.fl.metrics import (confusion_matrix, mean_over_clients, metrics_from_confusion, pooled)

skm = pytest.importorskip("sklearn.metrics")


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("C", [2, 3, 5])
def test_metrics_match_sklearn(seed, C):
    rng = np.random.RandomState(seed)
    n = rng.randint(5, 300)
    y = rng.randint(0, C, n)
    p = rng.randint(0, C if seed % 2 else 1, n)   # sometimes degenerate predictions
    m = metrics_from_confusion(confusion_matrix(y, p, C))
    ref = {
        "accuracy": skm.accuracy_score(y, p),
        "precision": skm.precision_score(y, p, average="weighted", zero_division=0),
        "recall": skm.recall_score(y, p, average="weighted", zero_division=0),
        "f1": skm.f1_score(y, p, average="weighted", zero_division=0),
    }
    for k in ref:
        assert abs(m[k] - ref[k]) < 1e-12, (k, m[k], ref[k])


def test_weighted_recall_equals_accuracy():
    y = np.array([0, 0, 1, 1, 1]); p = np.array([0, 1, 1, 1, 0])
    m = metrics_from_confusion(confusion_matrix(y, p, 2))
    assert m["recall"] == m["accuracy"]


def test_pooled_equals_concatenated():
    rng = np.random.RandomState(1)
    ys = [rng.randint(0, 2, 40) for _ in range(3)]
    ps = [rng.randint(0, 2, 40) for _ in range(3)]
    cms = [confusion_matrix(a, b, 2) for a, b in zip(ys, ps)]
    ref = metrics_from_confusion(confusion_matrix(np.concatenate(ys), np.concatenate(ps), 2))
    assert pooled(cms) == ref
    mean = mean_over_clients([metrics_from_confusion(c) for c in cms])
    assert abs(mean["accuracy"] - np.mean([metrics_from_confusion(c)["accuracy"] for c in cms])) < 1e-15


def _reference_rule(seq, patience=10, tol=1e-4):
    """Literal transcription of C:181-192 (rank-0 branch)."""
    termination_count = patience
    prev_metric = None
    for r, avg in enumerate(seq):
        if prev_metric is not None and np.allclose(avg, prev_metric, atol=tol):
            termination_count -= 1
            if termination_count == 0:
                return r
        else:
            prev_metric = avg
            termination_count = patience
    return None


@pytest.mark.parametrize("seed", range(20))
def test_early_stop_oracle(seed):
    rng = np.random.RandomState(seed)
    seq, v = [], rng.rand(4)
    for _ in range(200):
        if rng.rand() < 0.3:
            v = v + rng.randn(4) * 1e-3
        else:
            v = v + rng.randn(4) * 2e-5
        seq.append(v.copy())
    es = EarlyStopper(patience=5, tolerance=1e-4)
    got = None
    for r, x in enumerate(seq):
        if es.update(x):
            got = r
            break
    assert got == _reference_rule(seq, patience=5)


def test_allclose_rtol_matches_numpy():
    a = np.array([1.0, 0.5, 0.2, 0.9]); b = a + 1.04e-4
    assert allclose(a, b, 1e-4) == np.allclose(a, b, atol=1e-4)
