"""Synthetic income-shaped tabular data.

The north star benchmarks on *synthetic balanced-income-shaped* rows (BASELINE.json): 14
standardised features -- 6 heavy-tailed "integer" columns and 8 label-encoded categorical
columns with the cardinalities of ``balanced_income_data.csv`` -- and a
balanced binary label produced by a fixed random teacher so that accuracy is meaningful.

Two generators with the same distribution:

* :func:`make_income_like` -- numpy, for CPU tests and small shards;
* :func:`make_income_like_device` -- the HIP Philox kernel (``synth_income`` in
  ``fedmi/ops/csrc/fl_kernels.hip``) that writes a shard straight into device memory, so a
  1e8-row shard never crosses PCIe.
"""
from __future__ import annotations

import numpy as np

# cardinalities of the 8 categorical columns of the income table
CAT_CARDINALITY = (7, 16, 7, 14, 6, 5, 2, 40)
N_NUMERIC = 6
N_FEATURES = N_NUMERIC + len(CAT_CARDINALITY)  # 14


def teacher_weights(seed: int = 1234, n_features: int = N_FEATURES, hidden: int = 16):
    rng = np.random.RandomState(seed)
    w1 = rng.standard_normal((hidden, n_features)).astype(np.float32) / np.sqrt(n_features)
    w2 = rng.standard_normal(hidden).astype(np.float32) / np.sqrt(hidden)
    return w1, w2


def make_income_like(n: int, seed: int = 0, teacher_seed: int = 1234, dtype=np.float32):
    """Return ``(X [n,14], y [n])`` with a balanced label (teacher score vs its median 0)."""
    rng = np.random.RandomState(seed)
    num = rng.standard_normal((n, N_NUMERIC))
    num[:, 2] = np.expm1(np.abs(num[:, 2]))          # fnlwgt-like heavy tail
    num[:, 3] = np.where(rng.rand(n) < 0.9, 0.0, np.abs(num[:, 3]) * 3)  # capital.gain-like
    cats = [rng.randint(0, c, size=n) for c in CAT_CARDINALITY]
    cat = np.stack(cats, axis=1).astype(np.float64)
    cat = (cat - cat.mean(0)) / np.maximum(cat.std(0), 1e-12)
    num = (num - num.mean(0)) / np.maximum(num.std(0), 1e-12)
    X = np.concatenate([num, cat], axis=1).astype(dtype)
    w1, w2 = teacher_weights(teacher_seed)
    score = np.maximum(X.astype(np.float32) @ w1.T, 0.0) @ w2
    y = (score > np.median(score)).astype(np.int64)
    return X, y


# label noise of the device shards: the income table's best accuracies are ~0.84-0.86, so the
# synthetic task flips 15 % of the teacher's labels (Bayes accuracy 0.85) instead of being
# separable
DEVICE_LABEL_NOISE = 0.15


def device_shard(n_rows: int, rank: int, device, seed: int = 7, label_noise: float = DEVICE_LABEL_NOISE):
    """Income-shaped rows generated ON the device by the Philox kernel (no host copy; the
    1e8-row shards of BASELINE config 3): client ``rank`` gets rows
    ``[rank * n_rows, (rank + 1) * n_rows)`` of one global counter-based stream, labels from
    the same teacher as :func:`make_income_like`, balanced by a threshold estimated on a host
    sample of the same distribution, each flipped with probability ``label_noise``."""
    import torch
    from ..ops import native
    if n_rows <= 0:
        raise ValueError(f"device_shard needs n_rows > 0 (got {n_rows})")
    m = native()
    w1, w2 = teacher_weights()
    Xs, _ = make_income_like(4096, seed=123)
    th = float(np.median(np.maximum(Xs @ w1.T, 0.0) @ w2))
    X = torch.empty((n_rows, N_FEATURES), dtype=torch.float32, device=device)
    y = torch.empty(n_rows, dtype=torch.int32, device=device)
    tw1 = torch.as_tensor(w1, device=device)
    tw2 = torch.as_tensor(np.append(w2, th).astype(np.float32), device=device)
    m.synth(X.data_ptr(), y.data_ptr(), n_rows, N_FEATURES, seed, rank * n_rows, tw1.data_ptr(), tw2.data_ptr(),
            int(w1.shape[0]), torch.cuda.current_stream(device).cuda_stream, float(label_noise))
    torch.cuda.synchronize(device)
    return X, y
