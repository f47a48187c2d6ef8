"""Host emulation of the early-stopping behaviour of bf16 training vs the scoring precision.

The reference's stop rule (``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:181-192``)
needs 10 consecutive rounds whose 4 metrics stay within atol 1e-4 of the last significant
value: on an 8000-row shard that means *no prediction flips* for 10 rounds.  This script
trains the [C] model (k = 1, compat mode, real CSV) with the bf16 kernels' rounding points
emulated in torch (bf16 weights / activations / deltas as MFMA operands, fp32 accumulation,
fp32 master weights and Adam) and scores each round's post-step model with

* ``bf16``   -- the same bf16 forward the fused kernels use for scoring,
* ``fp32``   -- an fp32 forward on the fp32 master weights,
* ``bf16x3`` -- split-bf16 forward (hi*hi + hi*lo + lo*hi, fp32 accumulate),

and prints the early-stop round and rounds-to-0.80/0.83 for each.  CPU only.

    python tools/bf16_es_emulate.py --seeds 0 1 2 3 4
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fedmi.data.sharding import split_data  # noqa: E402
from fedmi.data.tabular import load_tabular  # noqa: E402
from fedmi.fl.early_stop import EarlyStopper  # noqa: E402
from fedmi.fl.metrics import metric_vector, metrics_from_confusion, confusion_matrix  # noqa: E402
from fedmi.models.mlp import init_flat, flat_to_dict  # noqa: E402


def bf(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(torch.float32)


def split3_mm(a: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    ah, wh = bf(a), bf(w)
    al, wl = bf(a - ah), bf(w - wh)
    return ah @ wh.T + al @ wh.T + ah @ wl.T


def forward(Ws, bs, X, mode):
    a = X
    acts, pre = [a], []
    for l, (W, b) in enumerate(zip(Ws, bs)):
        if mode == "fp32":
            z = a @ W.T + b
        elif mode == "bf16x3":
            z = split3_mm(a, W) + b
        elif mode == "w2":      # bf16 activations, split-bf16 weights (hi + lo)
            ah, wh = bf(a), bf(W)
            z = ah @ wh.T + ah @ bf(W - wh).T + b
        elif mode == "a2":      # split-bf16 activations, bf16 weights
            ah, wh = bf(a), bf(W)
            z = ah @ wh.T + bf(a - ah) @ wh.T + b
        else:
            z = bf(a) @ bf(W).T + b
        pre.append(z)
        if l < len(Ws) - 1:
            a = torch.relu(z)
            if mode in ("bf16", "w2"):
                a = bf(a)
            acts.append(a)
    return z, acts, pre


def grads_bf16(Ws, bs, X, y, fwd="bf16"):
    """Gradient with the bf16 kernels' operand rounding (fp32 accumulation); ``fwd`` = the
    forward pass's precision (the backward always uses bf16 activations / deltas / weights)."""
    z, acts, pre = forward(Ws, bs, X, fwd)
    acts = [bf(t) for t in acts]
    n = X.shape[0]
    p = torch.softmax(z, 1)
    loss = -torch.log(p[torch.arange(n), y]).mean()
    d = p.clone()
    d[torch.arange(n), y] -= 1.0
    d /= n
    gW, gb = [None] * len(Ws), [None] * len(Ws)
    for l in range(len(Ws) - 1, -1, -1):
        db = bf(d)
        gW[l] = db.T @ bf(acts[l])
        gb[l] = d.sum(0)
        if l:
            da = db @ bf(Ws[l])
            d = da * (pre[l - 1] > 0)
    return gW, gb, float(loss)


def grads_fp32(Ws, bs, X, y):
    params = [t.clone().requires_grad_(True) for t in Ws + bs]
    L = len(Ws)
    a = X
    for l in range(L):
        a = a @ params[l].T + params[L + l]
        if l < L - 1:
            a = torch.relu(a)
    loss = torch.nn.functional.cross_entropy(a, y)
    loss.backward()
    return [p.grad for p in params[:L]], [p.grad for p in params[L:]], float(loss)


def run(seed: int, train: str, score_modes, rounds: int = 300):
    ds = load_tabular()
    X, y = split_data(ds.X_train, ds.y_train, 0, 1, mode="compat", seed=seed)
    X = torch.as_tensor(np.asarray(X, np.float32))
    y = torch.as_tensor(np.asarray(y), dtype=torch.long)
    dims = [14, 50, 200, 2]
    d = flat_to_dict(init_flat(dims, seed * 1000003), dims)
    L = len(dims) - 1
    Ws = [torch.as_tensor(d[f"model.{2 * l}.weight"]).clone() for l in range(L)]
    bs = [torch.as_tensor(d[f"model.{2 * l}.bias"]).clone() for l in range(L)]
    params = Ws + bs
    m = [torch.zeros_like(p) for p in params]
    v = [torch.zeros_like(p) for p in params]
    b1, b2, eps = 0.9, 0.999, 1e-8
    stoppers = {k: EarlyStopper() for k in score_modes}
    out = {k: {"stop": None, "0.80": None, "0.83": None} for k in score_modes}
    for r in range(rounds):
        if train == "fp32":
            gW, gb, _ = grads_fp32(Ws, bs, X, y)
        else:
            gW, gb, _ = grads_bf16(Ws, bs, X, y, {"bf16": "bf16", "bf16w2": "w2", "bf16x3": "bf16x3"}[train])
        lr = 0.004 * 0.5 ** (r // 30)
        t = r + 1
        for i, (p, g) in enumerate(zip(params, gW + gb)):
            m[i].mul_(b1).add_(g, alpha=1 - b1)
            v[i].mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v[i].sqrt() / (1 - b2 ** t) ** 0.5).add_(eps)
            p.addcdiv_(m[i], denom, value=-lr / (1 - b1 ** t))
        for k in score_modes:
            if out[k]["stop"] is not None:
                continue
            z, _, _ = forward(Ws, bs, X, k)
            cm = confusion_matrix(y.numpy(), z.argmax(1).numpy(), 2)
            g = metric_vector(metrics_from_confusion(cm))
            for tgt in ("0.80", "0.83"):
                if out[k][tgt] is None and g[0] >= float(tgt):
                    out[k][tgt] = r + 1
            if stoppers[k].update(g):
                out[k]["stop"] = r + 1
                out[k]["final_acc"] = float(g[0])
        if all(out[k]["stop"] is not None for k in score_modes):
            break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--train", nargs="+", default=["fp32", "bf16"], help="fp32 | bf16 | bf16w2 | bf16x3 (bf16 backward, forward in the named precision)")
    ap.add_argument("--score", nargs="+", default=None)
    a = ap.parse_args()
    torch.set_num_threads(1)
    for tr in a.train:
        modes = a.score or (["fp32"] if tr == "fp32" else ["bf16", "fp32", "bf16x3", "w2", "a2"])
        for s in a.seeds:
            res = run(s, tr, modes)
            print(f"train={tr} seed={s} " + " ".join(f"score={k}:{res[k]}" for k in modes), flush=True)


if __name__ == "__main__":
    main()
