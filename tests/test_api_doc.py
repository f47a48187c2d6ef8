"""docs/API.md's examples, on the CPU backends (one client, no communicator): the API a user of the
reference switches to stays what the document says."""
import warnings

import numpy as np

from fedmi.data.tabular import load_tabular
from fedmi.fl.engine import EngineConfig
from fedmi.fl.sklearn_fed import allreduce_confusion, average_estimator_weights
from fedmi.fl.trainer import FederatedMLPLearning
from fedmi.hpo.sweep import run_sweep
from fedmi.models.sklearn_mlp import MLPClassifier, fit_packed


def test_c_trainer_example():
    ds = load_tabular(with_mean=True)
    cfg = EngineConfig(early_stop=True, patience=10, tolerance=1e-4)
    fl = FederatedMLPLearning(ds.X_train, ds.y_train, 0, 1, comm=None, hidden_sizes=[50, 200], config=cfg,
                              backend="torch")
    hist = fl.train_and_evaluate(None, rounds=3, verbose=False)
    assert sorted(hist) == ["accuracy", "f1", "precision", "recall"] and len(hist["accuracy"]) == 3
    test = fl.evaluate_global(ds.X_test, ds.y_test, None)
    assert 0.5 < test["accuracy"] <= 1.0
    w = fl.get_weights()
    assert list(w) == ["model.0.weight", "model.0.bias", "model.2.weight", "model.2.bias",
                       "model.4.weight", "model.4.bias"]
    assert w["model.0.weight"].shape == (50, 14)
    fl.set_weights(w)
    for name in ("_split_data", "train_one_epoch", "evaluate_local", "federated_averaging"):
        assert callable(getattr(fl, name))


def test_sklearn_examples():
    warnings.filterwarnings("ignore")
    ds = load_tabular(with_mean=False)
    X, y = ds.X_train[:600], ds.y_train[:600]
    clf = MLPClassifier(hidden_layer_sizes=(50, 400), learning_rate_init=0.004, max_iter=3, random_state=42,
                        backend="numpy")
    clf.fit(X, y)
    assert clf.predict_proba(X).shape == (600, 2) and 0.0 <= clf.score(X, y) <= 1.0
    assert [c.shape for c in clf.coefs_] == [(14, 50), (50, 400), (400, 1)]
    assert len(average_estimator_weights(clf, None)) == 6
    cm = np.array([[3, 1], [0, 4]])
    assert (allreduce_confusion(cm, None) == cm).all()
    ests = [MLPClassifier(hidden_layer_sizes=(20,), learning_rate_init=lr, max_iter=3, random_state=42,
                          backend="numpy") for lr in (0.002, 0.01)]
    fit_packed(ests, X, y)
    assert all(e.n_iter_ == 3 for e in ests)
    best, res = run_sweep(X, y, None, [(5,), (8,)], [0.01, 0.02], max_iter=3, backend="numpy")
    assert len(res) == 4 and best in res
