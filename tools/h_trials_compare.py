"""Per-trial comparison of [H] sweeps: the HIP sweep's `sweep.json` (hyperparameters_tuning.py --save) against
scikit-learn fits of the same grid (tools/h_trials_sklearn.py), and scikit-learn against itself at another BLAS
thread count.  Pooled training accuracy at k = 1 is the reference's global metric (hyperparameters_tuning.py:105-118).

    python tools/h_trials_compare.py --hip gpurun_out/h_trials_hip_r6.json \
        --sk profiles/h_trials_sklearn_1thr.json [--sk2 profiles/h_trials_sklearn_8thr.json]
"""
import argparse
import json

import numpy as np


def _load_hip(path):
    with open(path) as f:
        d = json.load(f)
    return {(tuple(t["hidden"]), float(t["lr"])): (float(t["global"]["accuracy"]), int(t["n_iter"]))
            for t in d["trials"]}


def _load_sk(path):
    with open(path) as f:
        d = json.load(f)
    return {(tuple(t["hidden"]), float(t["lr"])): (float(t["accuracy"]), int(t["n_iter"])) for t in d["trials"]}


def _ranks(v):
    return np.argsort(np.argsort(v)).astype(np.float64)


def compare(a, b, name_a, name_b, table=False):
    keys = sorted(set(a) & set(b), key=lambda k: (sum(k[0]), k[0], k[1]))
    da = np.array([a[k][0] for k in keys])
    db = np.array([b[k][0] for k in keys])
    na = np.array([a[k][1] for k in keys])
    nb = np.array([b[k][1] for k in keys])
    diff = np.abs(da - db)
    rho = float(np.corrcoef(_ranks(da), _ranks(db))[0, 1])
    ba = max(keys, key=lambda k: a[k][0])
    bb = max(keys, key=lambda k: b[k][0])
    out = []
    if table:
        out.append(f"# {'hidden':<11} {'lr':>6}  {name_a:>14} [n_iter]  {name_b:>14} [n_iter]  |d acc|")
        for k, x, y, m, n in zip(keys, da, db, na, nb):
            out.append(f"  {str(k[0]):<11} {k[1]:>6}  {x:>14.6f} [{m:>4}]  {y:>14.6f} [{n:>4}]  {abs(x - y):.5f}")
    out.append(f"{name_a} vs {name_b}: {len(keys)} trials; |d acc| mean {diff.mean():.5f} median "
               f"{np.median(diff):.5f} p90 {np.quantile(diff, 0.9):.5f} max {diff.max():.5f}; "
               f"same n_iter {int((na == nb).sum())}/{len(keys)}; |d n_iter| median {np.median(np.abs(na - nb)):.0f}; "
               f"Spearman rho {rho:.3f}")
    out.append(f"  best {name_a}: {ba[0]} lr {ba[1]} -> {a[ba][0]:.6f} ({name_b} there: {b[ba][0]:.6f}); "
               f"best {name_b}: {bb[0]} lr {bb[1]} -> {b[bb][0]:.6f} ({name_a} there: {a[bb][0]:.6f})")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hip", required=True)
    ap.add_argument("--sk", required=True)
    ap.add_argument("--sk2")
    a = ap.parse_args()
    hip, sk = _load_hip(a.hip), _load_sk(a.sk)
    print(compare(hip, sk, "hip_f64", "sklearn", table=True))
    if a.sk2:
        sk2 = _load_sk(a.sk2)
        print(compare(sk2, sk, "sklearn_2", "sklearn"))
        print(compare(hip, sk2, "hip_f64", "sklearn_2"))


if __name__ == "__main__":
    main()
