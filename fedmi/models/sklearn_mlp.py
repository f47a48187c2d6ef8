"""scikit-learn-compatible ``MLPClassifier`` on fedmi kernels (native component N9).

The [S] and [H] reference scripts train ``sklearn.neural_network.MLPClassifier``
(``FL_SkLearn_MLPClassifier_Limitation.py:77-101``, ``hyperparameters_tuning.py:90-91``).
This estimator keeps that API -- ``fit``, ``partial_fit``, ``predict``, ``predict_proba``,
``score``, ``coefs_`` / ``intercepts_`` ([in, out], float64), ``n_iter_``, ``loss_``,
``loss_curve_``, ``best_loss_``, ``t_``, ``classes_`` -- and sklearn's training algorithm:

* Glorot-uniform init ``U(+-sqrt(6 / (fan_in + fan_out)))`` drawn from
  ``RandomState(random_state)`` in sklearn's order, re-created at every ``fit`` call
  (which is why ``fit`` after ``_set_weights`` discards the averaged model: SURVEY Q8);
* logistic output + binary log-loss for two classes, softmax + log-loss otherwise;
* L2 penalty ``alpha`` on the coefficients (gradient ``(dW + alpha W) / batch``, loss
  ``+ 0.5 alpha sum W^2 / batch``);
* sklearn's Adam (``lr_t = lr sqrt(1-b2^t) / (1-b1^t)``, ``-lr_t m / (sqrt(v) + eps)``);
* minibatches of ``min(200, n)`` rows, reshuffled every epoch from the same RandomState;
* stop after ``n_iter_no_change`` epochs without a ``tol`` improvement of the training loss.

Backends: ``"hip"`` trains on the device with the native packed-trial trainer
(``MLPTrainer`` / ``MLPTrainer64`` in ``fedmi/ops/csrc/mlp_trainer.cpp``: fused-epilogue MFMA
GEMMs, device-side loss / Adam / stop rule, one HIP-graph launch per epoch) in
``dtype="float64"`` (the default, sklearn's own precision: ``v_mfma_f64_16x16x4_f64`` GEMMs of
``mlp_f64.hip``) or ``dtype="float32"`` (exact-fp32 MFMA); ``"numpy"`` is a float64 host
implementation of the same algorithm (the CPU path and the parity oracle -- it tracks
sklearn to ~1e-12).  ``warm_start=True`` fixes the reference's limitation: a ``fit`` after
``_set_weights`` continues from the averaged weights.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np


def _glorot(rs: np.random.RandomState, dims: Sequence[int]):
    coefs, inters = [], []
    for fan_in, fan_out in zip(dims[:-1], dims[1:]):
        bound = np.sqrt(6.0 / (fan_in + fan_out))
        coefs.append(rs.uniform(-bound, bound, (fan_in, fan_out)))
        inters.append(rs.uniform(-bound, bound, fan_out))
    return coefs, inters


def epoch_permutations(rs: np.random.RandomState, n: int, epochs: int) -> np.ndarray:
    """sklearn's per-epoch ``sample_idx = shuffle(sample_idx, random_state=rs)`` sequence.  With the
    native extension the same MT19937 draws run in C++ without the GIL (sk_perms.cpp: numpy's
    generator, state in / state out, bit for bit), so packed jobs prepare their orders concurrently."""
    st = rs.get_state() if isinstance(rs, np.random.RandomState) else None
    if st is not None and st[0] == "MT19937" and epochs > 0 and n > 0:
        try:
            from ..ops import native, native_available
            m = native() if native_available() else None
        except Exception:  # noqa: BLE001 -- the numpy loop below is the reference
            m = None
        if m is not None and hasattr(m, "sk_epoch_perms"):
            perms, key, pos = m.sk_epoch_perms(st[1], int(st[2]), int(n), int(epochs))
            rs.set_state((st[0], key, pos, st[3], st[4]))
            return perms
    out = np.empty((epochs, n), dtype=np.int32)
    idx = np.arange(n)
    for e in range(epochs):
        ind = np.arange(n)
        rs.shuffle(ind)
        idx = idx[ind]
        out[e] = idx
    return out


def _relu(x):
    return np.maximum(x, 0)


def _softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def _logistic(z):
    from scipy.special import expit
    return expit(z)


class MLPClassifier:
    """Drop-in for ``sklearn.neural_network.MLPClassifier`` (relu / adam subset)."""

    def __init__(self, hidden_layer_sizes=(100,), activation="relu", solver="adam", alpha=1e-4,
                 batch_size="auto", learning_rate_init=1e-3, max_iter=200, shuffle=True, random_state=None,
                 tol=1e-4, verbose=False, warm_start=False, beta_1=0.9, beta_2=0.999, epsilon=1e-8,
                 n_iter_no_change=10, backend="auto", device=None, dtype="float64"):
        if activation != "relu" or solver != "adam":
            raise NotImplementedError("fedmi MLPClassifier supports activation='relu', solver='adam'")
        self.hidden_layer_sizes = hidden_layer_sizes
        self.activation = activation
        self.solver = solver
        self.alpha = alpha
        self.batch_size = batch_size
        self.learning_rate_init = learning_rate_init
        self.max_iter = max_iter
        self.shuffle = shuffle
        self.random_state = random_state
        self.tol = tol
        self.verbose = verbose
        self.warm_start = warm_start
        self.beta_1 = beta_1
        self.beta_2 = beta_2
        self.epsilon = epsilon
        self.n_iter_no_change = n_iter_no_change
        self.backend = backend
        self.device = device
        dtype = {"fp64": "float64", "fp32": "float32"}.get(dtype, dtype)
        if dtype not in ("float64", "float32"):
            raise ValueError("dtype must be 'float64' (fp64) or 'float32' (fp32)")
        self.dtype = dtype

    # ------------------------------------------------------------------ helpers
    def _resolve_backend(self) -> str:
        if self.backend != "auto":
            return self.backend
        try:
            import torch
            return "hip" if torch.cuda.is_available() else "numpy"
        except Exception:
            return "numpy"

    def _rs(self) -> np.random.RandomState:
        rs = self.random_state
        if rs is None:
            return np.random.mtrand._rand
        if isinstance(rs, np.random.RandomState):
            return rs
        return np.random.RandomState(rs)

    def _dims(self, n_features: int) -> List[int]:
        h = self.hidden_layer_sizes
        h = list(h) if hasattr(h, "__iter__") else [h]
        return [n_features, *[int(x) for x in h], self.n_outputs_]

    def _encode(self, y, fit_classes: bool, classes=None):
        y = np.asarray(y)
        if fit_classes:
            self.classes_ = np.unique(y if classes is None else np.asarray(classes))
            if len(self.classes_) < 2:
                raise ValueError("need at least 2 classes")
            self.n_outputs_ = 1 if len(self.classes_) == 2 else len(self.classes_)
            self.out_activation_ = "logistic" if self.n_outputs_ == 1 else "softmax"
        codes = np.searchsorted(self.classes_, y)
        if np.any(self.classes_[np.clip(codes, 0, len(self.classes_) - 1)] != y):
            raise ValueError("y contains classes not seen in the first fit")
        return codes.astype(np.int64)

    def _batch(self, n: int) -> int:
        return min(200, n) if self.batch_size == "auto" else int(np.clip(self.batch_size, 1, n))

    # ------------------------------------------------------------------ API
    def fit(self, X, y):
        return self._fit(X, y, incremental=False)

    def partial_fit(self, X, y, classes=None):
        return self._fit(X, y, incremental=True, classes=classes)

    def _fit(self, X, y, incremental: bool, classes=None):
        X = np.asarray(X, dtype=np.float64)
        first_pass = not hasattr(self, "coefs_") or (not self.warm_start and not incremental)
        if first_pass and not (incremental and hasattr(self, "classes_") and classes is None):
            codes = self._encode(y, True, classes)
        else:
            codes = self._encode(y, False)
        rs = self._rs()
        dims = self._dims(X.shape[1])
        if first_pass:
            self.coefs_, self.intercepts_ = _glorot(rs, dims)
            self.n_iter_ = 0
            self.t_ = 0
            self.n_layers_ = len(dims)
            self.loss_curve_ = []
            self._no_improvement_count = 0
            self.best_loss_ = np.inf
        if not incremental or not hasattr(self, "_adam"):
            self._adam = None    # fresh optimizer state (sklearn re-creates it on fit)
        epochs = 1 if incremental else self.max_iter
        perms = epoch_permutations(rs, X.shape[0], epochs) if self.shuffle else \
            np.tile(np.arange(X.shape[0], dtype=np.int32), (epochs, 1))
        backend = self._resolve_backend()
        if backend == "hip":
            _fit_hip([self], X, codes, dims, perms, incremental)
        else:
            _fit_numpy(self, X, codes, perms, incremental)
        return self

    def _forward(self, X):
        a = np.asarray(X, dtype=np.float64)
        L = len(self.coefs_)
        for i, (W, b) in enumerate(zip(self.coefs_, self.intercepts_)):
            a = a @ W + b
            if i < L - 1:
                a = _relu(a)
        return _logistic(a) if self.out_activation_ == "logistic" else _softmax(a)

    def predict_proba(self, X):
        p = self._forward(X)
        if self.n_outputs_ == 1:
            p = p.ravel()
            return np.stack([1 - p, p], axis=1)
        return p

    def predict(self, X):
        p = self._forward(X)
        if self.n_outputs_ == 1:
            return self.classes_[(p.ravel() > 0.5).astype(int)]
        return self.classes_[np.argmax(p, axis=1)]

    def score(self, X, y):
        return float(np.mean(self.predict(X) == np.asarray(y)))

    def get_params(self, deep=True):
        keys = ["hidden_layer_sizes", "activation", "solver", "alpha", "batch_size", "learning_rate_init",
                "max_iter", "shuffle", "random_state", "tol", "verbose", "warm_start", "beta_1", "beta_2",
                "epsilon", "n_iter_no_change", "backend", "device", "dtype"]
        return {k: getattr(self, k) for k in keys}


# ---------------------------------------------------------------------- numpy (fp64)
class _AdamState:
    def __init__(self, params):
        self.t = 0
        self.ms = [np.zeros_like(p) for p in params]
        self.vs = [np.zeros_like(p) for p in params]


def _fit_numpy(est: MLPClassifier, X, codes, perms, incremental):
    n = X.shape[0]
    B = est._batch(n)
    params = est.coefs_ + est.intercepts_
    if est._adam is None:
        est._adam = _AdamState(params)
    opt = est._adam
    L = len(est.coefs_)
    if est.n_outputs_ == 1:
        Y = codes.reshape(-1, 1).astype(np.float64)
    else:
        Y = np.eye(est.n_outputs_)[codes]
    eps = np.finfo(np.float64).eps
    for e in range(perms.shape[0]):
        idx = perms[e]
        acc = 0.0
        for s in range(0, n, B):
            bi = idx[s:s + B]
            xb, yb = X[bi], Y[bi]
            m = len(bi)
            acts = [xb]
            for i in range(L):
                z = acts[-1] @ est.coefs_[i] + est.intercepts_[i]
                acts.append(_relu(z) if i < L - 1 else (_logistic(z) if est.n_outputs_ == 1 else _softmax(z)))
            p = np.clip(acts[-1], eps, 1 - eps)
            if est.n_outputs_ == 1:
                loss = -np.mean(yb * np.log(p) + (1 - yb) * np.log(1 - p)) * 1.0
                loss = float(np.sum(loss))
            else:
                loss = float(-np.sum(yb * np.log(p)) / m)
            loss += 0.5 * est.alpha * sum(float(np.dot(c.ravel(), c.ravel())) for c in est.coefs_) / m
            delta = acts[-1] - yb
            cg, ig = [None] * L, [None] * L
            for i in range(L - 1, -1, -1):
                cg[i] = (acts[i].T @ delta + est.alpha * est.coefs_[i]) / m
                ig[i] = delta.mean(axis=0)
                if i > 0:
                    delta = (delta @ est.coefs_[i].T) * (acts[i] > 0)
            acc += loss * m
            grads = cg + ig
            opt.t += 1
            lr = est.learning_rate_init * np.sqrt(1 - est.beta_2 ** opt.t) / (1 - est.beta_1 ** opt.t)
            for k, (pk, g) in enumerate(zip(params, grads)):
                opt.ms[k] = est.beta_1 * opt.ms[k] + (1 - est.beta_1) * g
                opt.vs[k] = est.beta_2 * opt.vs[k] + (1 - est.beta_2) * g * g
                pk += -lr * opt.ms[k] / (np.sqrt(opt.vs[k]) + est.epsilon)
        est.n_iter_ += 1
        est.loss_ = acc / n
        est.t_ += n
        est.loss_curve_.append(est.loss_)
        if est.loss_curve_[-1] > est.best_loss_ - est.tol:
            est._no_improvement_count += 1
        else:
            est._no_improvement_count = 0
        if est.loss_curve_[-1] < est.best_loss_:
            est.best_loss_ = est.loss_curve_[-1]
        if est._no_improvement_count > est.n_iter_no_change:
            break
        if incremental:
            break


# ---------------------------------------------------------------------- HIP (packed)
def _pack(coefs, inters, dtype=np.float32) -> np.ndarray:
    parts = []
    for W, b in zip(coefs, inters):
        parts.append(np.asarray(W, dtype=dtype).T.reshape(-1))
        parts.append(np.asarray(b, dtype=dtype).reshape(-1))
    return np.concatenate(parts)


def _pack_t(coefs, inters) -> np.ndarray:
    """float64 flat layout of _pack with each layer's weights TRANSPOSED -- sklearn's own [in, out]
    = [K][N] -- at the same offsets (biases unused)."""
    parts = []
    for W, b in zip(coefs, inters):
        parts.append(np.asarray(W, dtype=np.float64).reshape(-1))
        parts.append(np.zeros(np.asarray(b).size, np.float64))
    return np.concatenate(parts)


def _unpack(flat, dims):
    coefs, inters, off = [], [], 0
    for K, N in zip(dims[:-1], dims[1:]):
        coefs.append(flat[off:off + N * K].reshape(N, K).T.astype(np.float64).copy())
        off += N * K
        inters.append(flat[off:off + N].astype(np.float64).copy())
        off += N
    return coefs, inters


def _fit_hip(ests: List[MLPClassifier], X, codes, dims, perms, incremental):
    _fit_hip_prepare(ests, X, codes, dims, perms, incremental).run().finish()


def _fit_hip_prepare(ests: List[MLPClassifier], X, codes, dims, perms, incremental) -> "_HipJob":
    """Train T estimators of one architecture (same data, same permutations) at once."""
    import torch
    from ..ops import native
    m = native()
    e0 = ests[0]
    T = len(ests)
    dev = torch.device("cuda", torch.cuda.current_device()) if e0.device is None else torch.device(e0.device)
    n, F = X.shape
    B = e0._batch(n)
    P = sum(a * b + b for a, b in zip(dims[:-1], dims[1:]))
    maxw = max(dims[1:])
    L = len(dims) - 1
    f64 = getattr(e0, "dtype", "float64") == "float64"
    npdt, tdt = (np.float64, torch.float64) if f64 else (np.float32, torch.float32)
    f32 = dict(dtype=tdt, device=dev)     # element type of every float buffer of the trainer
    params = torch.as_tensor(np.stack([_pack(e.coefs_, e.intercepts_, npdt) for e in ests]),
                             device=dev).contiguous()
    if e0._adam is None or not isinstance(e0._adam, dict) or T > 1 or e0._adam["m"].dtype != tdt:
        mom = torch.zeros(T, P, **f32)
        vel = torch.zeros(T, P, **f32)
        step = torch.zeros(T, dtype=torch.int64, device=dev)
    else:
        mom, vel, step = e0._adam["m"], e0._adam["v"], e0._adam["step"]
    wd_mask = np.zeros(P, dtype=np.uint8)
    off = 0
    for K, N in zip(dims[:-1], dims[1:]):
        wd_mask[off:off + N * K] = 1
        off += N * K + N
    max_iter = perms.shape[0]
    bufs_t = {
        "X": torch.as_tensor(np.ascontiguousarray(X, npdt), device=dev),
        "y": torch.as_tensor(codes.astype(np.int32), device=dev),
        "perms": torch.as_tensor(np.ascontiguousarray(perms, np.int32), device=dev),
        "epoch_ctr": torch.zeros(1, dtype=torch.int32, device=dev),
        "params": params, "grads": torch.zeros(T, P, **f32), "m": mom, "v": vel,
        "anchor": params, "wd_mask": torch.as_tensor(wd_mask, device=dev),
        "lr": torch.as_tensor([float(e.learning_rate_init) for e in ests], dtype=torch.float64, device=dev),
        "step": step,
        "loss_acc": torch.zeros(T, dtype=torch.float64, device=dev),
        "best": torch.as_tensor([float(e.best_loss_) for e in ests], dtype=torch.float64, device=dev),
        "count": torch.as_tensor([int(e._no_improvement_count) for e in ests], dtype=torch.int32, device=dev),
        "n_iter": torch.zeros(T, dtype=torch.int32, device=dev),
        "active": torch.ones(T, dtype=torch.int32, device=dev),
        "curve": torch.zeros(T, max_iter, dtype=torch.float64, device=dev),
        # (the fused float64 step gathers each trial's rows into its own [B][F] slice)
        "xb": torch.zeros(T, B, F, **f32), "yb": torch.zeros(B, dtype=torch.int32, device=dev),
        "acts": torch.zeros(L, T, B, maxw, **f32), "deltas": torch.zeros(L, T, B, maxw, **f32),
    }
    cfg = {"n_rows": n, "batch": B, "head": 1 if e0.n_outputs_ == 1 else 0, "style": 1,
           "beta1": float(e0.beta_1), "beta2": float(e0.beta_2), "eps": float(e0.epsilon),
           "alpha": float(e0.alpha), "weight_decay": 0.0, "mu": 0.0, "tol": float(e0.tol),
           "n_iter_no_change": int(e0.n_iter_no_change), "max_iter": max_iter,
           "tol_stop": 0 if incremental else 1, "maxw": maxw}
    if f64 and os.environ.get("FEDMI_SK_WT", "1") != "0":
        # each layer's weights also transposed ([K][N]): the fused step's forward reads whole cache
        # lines of them (mlp_fused_f64.hip SkfArgs::wt); its Adam epilogue keeps them current
        wt = np.stack([_pack_t(e.coefs_, e.intercepts_) for e in ests])
        bufs_t["wt"] = torch.as_tensor(wt, device=dev).contiguous()
    trainer = m.MLPTrainer64 if f64 else m.MLPTrainer
    tr = trainer(list(dims), T, cfg, {k: v.data_ptr() for k, v in bufs_t.items()})
    for e in ests:
        e._hip_fused = bool(tr.fused)   # two-kernel minibatch step (mlp_fused_f64.hip) ran
        e._hip_split = int(getattr(tr, "split", 1))   # column slices of the row pass (skf_cs_*; 1 = none)
    stream = torch.cuda.Stream(device=dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    tr.prepare(stream.cuda_stream)      # the epoch graph, captured here (see _HipJob)
    return _HipJob(ests, tr, stream, dev, max_iter, bufs_t, params, mom, vel, step, dims, n, T)


class _HipJob:
    """A packed device fit in three steps: built and graph-captured (:func:`_fit_hip_prepare`),
    :meth:`run` (graph replays only: several jobs may run from several host threads at once),
    :meth:`finish` (results back into the estimators).  Building and capturing from one thread
    while no other thread issues HIP calls keeps every capture valid (the [H] sweep's threads)."""

    def __init__(self, ests, tr, stream, dev, max_iter, bufs_t, params, mom, vel, step, dims, n, T):
        self.ests, self.tr, self.stream, self.dev, self.max_iter = ests, tr, stream, dev, max_iter
        self.bufs_t, self.params, self.mom, self.vel, self.step = bufs_t, params, mom, vel, step
        self.dims, self.n, self.T = dims, n, T

    def run(self):
        import torch
        torch.cuda.set_device(self.dev)
        self.tr.run(self.max_iter, self.stream.cuda_stream, 8, True)
        self.stream.synchronize()
        return self

    def finish(self):
        ests, tr, bufs_t, params, dims, n, T = self.ests, self.tr, self.bufs_t, self.params, self.dims, self.n, self.T
        mom, vel, step = self.mom, self.vel, self.step
        _fit_hip_finish(ests, tr, bufs_t, params, mom, vel, step, dims, n, T)


def _fit_hip_finish(ests, tr, bufs_t, params, mom, vel, step, dims, n, T):
    if hasattr(tr, "stamps"):
        for e in ests:
            e._hip_stamps = list(tr.stamps())   # FEDMI_SK_STAMPS=1 (tools/sk_step_bench.py)
    flat = params.cpu().numpy()
    n_iter = bufs_t["n_iter"].cpu().numpy()
    curve = bufs_t["curve"].cpu().numpy()
    cnt = bufs_t["count"].cpu().numpy()
    best = bufs_t["best"].cpu().numpy()
    for t, e in enumerate(ests):
        e.coefs_, e.intercepts_ = _unpack(flat[t], dims)
        k = int(n_iter[t])
        e.loss_curve_.extend(float(x) for x in curve[t, :k])
        e.n_iter_ += k
        e.t_ += k * n
        e.loss_ = e.loss_curve_[-1] if e.loss_curve_ else None
        e.best_loss_ = float(best[t])
        e._no_improvement_count = int(cnt[t])
        if T == 1:
            e._adam = {"m": mom, "v": vel, "step": step}


def fit_packed(ests: List[MLPClassifier], X, y):
    """Fit several estimators that share architecture, data, random_state and batch size
    (e.g. the learning-rate axis of the [H] grid) as ONE packed device job."""
    job = prepare_packed(ests, X, y)
    if job is not None:
        job.run().finish()
    return ests


def prepare_packed(ests: List[MLPClassifier], X, y, inputs=None) -> Optional["_HipJob"]:
    """:func:`fit_packed` up to a built, graph-captured device job (None: a host backend, which
    has fitted the estimators already).  ``job.run()`` may then run beside other jobs from other
    host threads; ``job.finish()`` writes the results back."""
    X = np.asarray(X, dtype=np.float64)
    e0 = ests[0]
    sig = lambda e: (tuple(np.atleast_1d(e.hidden_layer_sizes)), e.random_state, e.batch_size, e.alpha,
                     e.max_iter, e.tol, e.n_iter_no_change, e.shuffle, getattr(e, "dtype", "float64"))
    if any(sig(e) != sig(e0) for e in ests):
        raise ValueError("fit_packed: estimators must share everything but learning_rate_init")
    if e0._resolve_backend() != "hip":
        for e in ests:
            e.fit(X, y)
        return None
    inputs = packed_inputs(ests, X, y) if inputs is None else inputs
    codes, perms = inputs
    return _fit_hip_prepare(ests, X, codes, e0._dims(X.shape[1]), perms, incremental=False)


def packed_inputs(ests: List[MLPClassifier], X, y):
    """The host half of :func:`prepare_packed`: every estimator's init (Glorot weights from its
    random_state) and the epochs' sample orders -- no HIP call, so several jobs may prepare theirs
    from several threads (the native order generator releases the GIL) before their device jobs are
    built and captured one after another."""
    X = np.asarray(X, dtype=np.float64)
    e0 = ests[0]
    rs, codes = None, None
    for e in ests:
        codes = e._encode(y, True)
        rs = e._rs()
        dims = e._dims(X.shape[1])
        e.coefs_, e.intercepts_ = _glorot(rs, dims)
        e.n_iter_, e.t_, e.n_layers_ = 0, 0, len(dims)
        e.loss_curve_, e._no_improvement_count, e.best_loss_ = [], 0, np.inf
        e._adam = None
    perms = epoch_permutations(rs, X.shape[0], e0.max_iter) if e0.shuffle else \
        np.tile(np.arange(X.shape[0], dtype=np.int32), (e0.max_iter, 1))
    return codes, perms
