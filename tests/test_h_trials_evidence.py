"""The committed [H] per-trial parity records (profiles/h_trials_*) say what README / convergence_r6.md claim.

The records come from a GPU run (hyperparameters_tuning.py --save) and CPU scikit-learn fits
(tools/h_trials_sklearn.py); this test re-reads them with tools/h_trials_compare.py's loaders.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
P = os.path.join(ROOT, "profiles")


def _pair(hip, sk):
    import h_trials_compare as hc
    a = hc._load_hip(os.path.join(P, hip))
    b = hc._load_sk(os.path.join(P, sk))
    assert set(a) == set(b) and len(a) == 90   # the reference grid: 10 hidden configs x 9 rates (H:73-74)
    return a, b


def test_k8_trials_equal_sklearn():
    a, b = _pair("h_trials_hip_k8_r6.json", "h_trials_sklearn_k8_1thr.json")
    assert all(a[k] == b[k] for k in a)          # pooled accuracy and epoch count, every trial
    best = max(a, key=lambda k: a[k][0])
    assert best == ((100, 400), 0.004) and a[best][0] == pytest.approx(0.967375)


def test_k1_trials_within_sklearns_own_spread():
    a, b = _pair("h_trials_hip_r6.json", "h_trials_sklearn_1thr.json")
    _, b2 = _pair("h_trials_hip_r6.json", "h_trials_sklearn_2thr.json")
    same = sum(a[k][0] == b[k][0] for k in a)
    self_same = sum(b2[k][0] == b[k][0] for k in a)
    assert same >= 75 and self_same >= 75
    worst = max(abs(a[k][0] - b[k][0]) for k in a)
    self_worst = max(abs(b2[k][0] - b[k][0]) for k in a)
    assert worst <= self_worst + 0.005


@pytest.mark.parametrize("k,best", [(2, ((100, 400), 0.004)), (4, ((100, 400), 0.002))])
def test_k2_k4_trials_equal_sklearn_but_one(k, best):
    a, b = _pair(f"h_trials_hip_k{k}_r6.json", f"h_trials_sklearn_k{k}_1thr.json")
    assert sum(a[k_][0] == b[k_][0] for k_ in a) >= 89
    assert max(a, key=lambda k_: a[k_][0]) == best == max(b, key=lambda k_: b[k_][0])
