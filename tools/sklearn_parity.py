"""[S] parity at k = 1/2/4/8 clients (BASELINE: pooled accuracy 0.954 / 0.953 / 0.957 / 0.941 at
round 5): every client fits MLPClassifier((50, 400), relu, lr 0.004, max_iter 300,
random_state 42) on its contiguous shard (partial_fit once, then fit -- the reference's call
sequence, S:77-101); the pooled metrics are the confusion matrices of the local predictions
summed over clients.  Because ``fit`` re-initialises the estimator (Q8), every round of the
reference repeats round 1, so round 5 == round 1 and the clients can be fitted one by one in
one process.

Fits, per shard: scikit-learn itself (the installed version, CPU) and fedmi's estimator on the
given backends (hip float64 = f64 MFMA trainer, hip float32, numpy float64); reports pooled
accuracy, epochs run and the agreement of each loss curve with sklearn's.

    python tools/sklearn_parity.py --backends hip:float64 hip:float32 --out profiles/sklearn_parity_r2.json
"""
import argparse
import json
import os
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--backends", nargs="+", default=["hip:float64", "hip:float32"])
    ap.add_argument("--no-sklearn", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    warnings.filterwarnings("ignore")
    from fedmi.data.sharding import split_data
    from fedmi.data.tabular import load_tabular
    from fedmi.fl.metrics import confusion_matrix, metrics_from_confusion
    from fedmi.models.sklearn_mlp import MLPClassifier
    ds = load_tabular(with_mean=False)
    kw = dict(activation="relu", hidden_layer_sizes=(50, 400), learning_rate_init=0.004, max_iter=300,
              random_state=42)
    makers = {}
    if not a.no_sklearn:
        import sklearn
        from sklearn.neural_network import MLPClassifier as SkMLP
        makers[f"sklearn-{sklearn.__version__}"] = lambda: SkMLP(**kw)
    for b in a.backends:
        be, dt = b.split(":")
        makers[b] = (lambda be=be, dt=dt: MLPClassifier(backend=be, dtype=dt, **kw))
    out = []
    for k in a.ks:
        row = {"k": k}
        curves = {}
        for name, make in makers.items():
            cm = np.zeros((2, 2), dtype=np.int64)
            iters, t0 = [], time.perf_counter()
            curves[name] = []
            for r in range(k):
                X, y = split_data(ds.X_train, ds.y_train, r, k, mode="contiguous")
                est = make()
                est.partial_fit(X, y, classes=np.unique(y))
                est.fit(X, y)
                cm += confusion_matrix(y, est.predict(X), 2)
                iters.append(int(est.n_iter_))
                curves[name].append(np.asarray(est.loss_curve_))
            m = metrics_from_confusion(cm)
            row[name] = {"pooled_accuracy": round(float(m["accuracy"]), 6), "n_iter": iters,
                         "wall_s": round(time.perf_counter() - t0, 3)}
            print(f"k={k} {name}: acc {m['accuracy']:.4f} n_iter {iters} ({row[name]['wall_s']} s)", flush=True)
        sk = [n for n in curves if n.startswith("sklearn")]
        if sk:
            ref = curves[sk[0]]
            for name in curves:
                if name == sk[0]:
                    continue
                agree = []   # epochs over which the loss curve tracks sklearn's to 1e-9 relative
                for c, s in zip(curves[name], ref):
                    n = min(len(c), len(s))
                    rel = np.abs(c[:n] - s[:n]) / np.abs(s[:n])
                    bad = np.nonzero(rel > 1e-9)[0]
                    agree.append(int(bad[0]) if len(bad) else n)
                row[name]["epochs_within_1e-9_of_sklearn"] = agree
        out.append(row)
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
