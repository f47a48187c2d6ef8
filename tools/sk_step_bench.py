"""Per-minibatch cost of the sklearn-compatible float64 trainer: fused two-kernel step
(mlp_fused_f64.hip) vs the layered path (FEDMI_SK_FUSED=0), on the [S] model (hidden (50, 400),
8000 rows, 200-row minibatches, 40 epochs = 1600 steps) and the [H] grid's largest packed job
((400, 200) x 9 learning rates).  Prints one JSON line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def run(hl, T, epochs, fused, X, y):
    from fedmi.models.sklearn_mlp import MLPClassifier, fit_packed
    os.environ["FEDMI_SK_FUSED"] = "1" if fused else "0"
    lrs = [0.002, 0.005, 0.004, 0.008, 0.01, 0.02, 0.05, 0.1, 0.2][:T]
    ests = [MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=lr, max_iter=epochs, random_state=42,
                          backend="hip", dtype="float64", tol=-1.0) for lr in lrs]
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fit_packed(ests, X, y)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = sum(e.n_iter_ for e in ests[:1]) * ((len(X) + 199) // 200)
    return {"hidden": list(hl), "trials": T, "epochs": int(ests[0].n_iter_), "fused": bool(ests[0]._hip_fused),
            "wall_s": dt, "us_per_step": dt / steps * 1e6, "final_loss": float(ests[0].loss_),
            "split": getattr(ests[0], "_hip_split", 1), "sk_split_env": os.environ.get("FEDMI_SK_SPLIT"),
            "stamps_us": [round(x, 2) for x in getattr(ests[0], "_hip_stamps", [])]}


def main():
    from fedmi.data.tabular import load_tabular
    ds = load_tabular(with_mean=False)
    X, y = ds.X_train, ds.y_train
    cases = [((50, 400), 1, 40), ((400, 200), 9, 10), ((50,), 9, 40), ((50, 400), 9, 20), ((400, 200), 1, 40),
             ((100, 400), 9, 20)]
    for i, arg in enumerate(sys.argv):
        if arg == "--case":
            cases = [cases[int(sys.argv[i + 1])]]
    modes = (True,) if "--fused-only" in sys.argv else (True, False)
    if "--stamps" in sys.argv:
        os.environ["FEDMI_SK_STAMPS"] = "1"
    for i, arg in enumerate(sys.argv):
        if arg == "--epochs":   # override every case's epoch count
            cases = [(hl, T, int(sys.argv[i + 1])) for hl, T, _ in cases]
    # --marginal: also fit 2x the epochs and report the marginal cost per step, (wall(2e) - wall(e)) /
    # (steps(2e) - steps(e)) -- free of the fit's set-up (trainer build, graph capture, copies), which
    # dominates short packed fits (10 epochs of 32 steps)
    marginal = "--marginal" in sys.argv
    for hl, T, ep in cases:
        run(hl, T, 2, True, X, y)   # warm-up (build, first graph)
        for fused in modes:
            r = run(hl, T, ep, fused, X, y)
            if marginal:
                r2 = run(hl, T, 2 * ep, fused, X, y)
                s1 = r["wall_s"] / r["us_per_step"] * 1e6
                s2 = r2["wall_s"] / r2["us_per_step"] * 1e6
                r["marginal_us_per_step"] = (r2["wall_s"] - r["wall_s"]) / max(s2 - s1, 1) * 1e6
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
