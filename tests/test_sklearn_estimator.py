"""fedmi MLPClassifier vs scikit-learn (float64 numpy backend: algorithmic parity), the
[S] limitation (Q8), warm-start fix, packed sweep semantics, and the HIP backends (float64 f64 MFMA, fp32)."""
import warnings

import numpy as np
import pytest

from fedmi.data.tabular import load_tabular
from fedmi.models.sklearn_mlp import MLPClassifier, epoch_permutations, fit_packed

sknn = pytest.importorskip("sklearn.neural_network")
warnings.filterwarnings("ignore")


@pytest.fixture(scope="module")
def data():
    ds = load_tabular(with_mean=False)
    return ds.X_train[:1500], ds.y_train[:1500]


@pytest.mark.parametrize("hl,mi", [((30,), 25), ((20, 40), 30), ((8, 8, 8), 20)])
def test_numpy_backend_matches_sklearn(data, hl, mi):
    X, y = data
    a = sknn.MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=0.004, max_iter=mi, random_state=42).fit(X, y)
    b = MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=0.004, max_iter=mi, random_state=42,
                      backend="numpy").fit(X, y)
    assert a.n_iter_ == b.n_iter_
    for u, v in zip(a.coefs_ + a.intercepts_, b.coefs_ + b.intercepts_):
        np.testing.assert_allclose(u, v, rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(a.loss_curve_, b.loss_curve_, rtol=1e-10)
    assert (a.predict(X) == b.predict(X)).all()
    np.testing.assert_allclose(a.predict_proba(X), b.predict_proba(X), atol=1e-9)


def test_multiclass_and_tol_stop_match_sklearn():
    rng = np.random.RandomState(0)
    X = rng.randn(400, 5)
    y = (X[:, 0] > 0).astype(int) + (X[:, 1] > 0.5).astype(int)     # 3 classes
    a = sknn.MLPClassifier(hidden_layer_sizes=(16,), learning_rate_init=0.01, max_iter=500, tol=1e-3,
                           random_state=3).fit(X, y)
    b = MLPClassifier(hidden_layer_sizes=(16,), learning_rate_init=0.01, max_iter=500, tol=1e-3, random_state=3,
                      backend="numpy").fit(X, y)
    assert a.n_iter_ == b.n_iter_ < 500          # stopped by the tol / n_iter_no_change rule
    np.testing.assert_allclose(a.loss_curve_, b.loss_curve_, rtol=1e-9)
    assert list(a.classes_) == list(b.classes_)


def test_partial_fit_then_fit_discards_weights_q8(data):
    """The [S] limitation: fit() re-initialises, so weights set before it are lost."""
    X, y = data
    m = MLPClassifier(hidden_layer_sizes=(10,), max_iter=5, random_state=42, backend="numpy")
    m.partial_fit(X, y, classes=np.unique(y))
    m.fit(X, y)
    ref = [c.copy() for c in m.coefs_]
    m.coefs_ = [np.zeros_like(c) for c in m.coefs_]           # "apply global weights"
    m.fit(X, y)
    for u, v in zip(ref, m.coefs_):
        np.testing.assert_array_equal(u, v)                     # identical: the averaged weights were discarded
    w = MLPClassifier(hidden_layer_sizes=(10,), max_iter=5, random_state=42, warm_start=True, backend="numpy")
    w.fit(X, y)
    w.coefs_ = [np.zeros_like(c) for c in w.coefs_]
    w.fit(X, y)
    assert not all(np.array_equal(u, v) for u, v in zip(ref, w.coefs_))


def test_epoch_permutations_follow_sklearn_rng():
    rs = np.random.RandomState(42)
    p = epoch_permutations(rs, 10, 3)
    from sklearn.utils import shuffle
    rs2 = np.random.RandomState(42)
    idx = np.arange(10)
    for e in range(3):
        idx = shuffle(idx, random_state=rs2)
        assert (p[e] == idx).all()


def test_fit_packed_cpu_equals_individual(data):
    X, y = data
    lrs = [0.002, 0.01]
    packed = [MLPClassifier(hidden_layer_sizes=(12,), learning_rate_init=lr, max_iter=8, random_state=42,
                            backend="numpy") for lr in lrs]
    fit_packed(packed, X, y)
    for lr, e in zip(lrs, packed):
        s = MLPClassifier(hidden_layer_sizes=(12,), learning_rate_init=lr, max_iter=8, random_state=42,
                          backend="numpy").fit(X, y)
        for u, v in zip(s.coefs_, e.coefs_):
            np.testing.assert_array_equal(u, v)


@pytest.mark.gpu
def test_hip_fp32_backend_tracks_float64(data):
    X, y = data
    a = MLPClassifier(hidden_layer_sizes=(50, 100), learning_rate_init=0.004, max_iter=15, random_state=42,
                      backend="numpy").fit(X, y)
    b = MLPClassifier(hidden_layer_sizes=(50, 100), learning_rate_init=0.004, max_iter=15, random_state=42,
                      backend="hip", dtype="float32").fit(X, y)
    assert b.n_iter_ == a.n_iter_
    np.testing.assert_allclose(b.loss_curve_[:5], a.loss_curve_[:5], rtol=2e-4)
    assert (a.predict(X) == b.predict(X)).mean() > 0.97


@pytest.mark.gpu
@pytest.mark.parametrize("hl,binary", [((50, 100), True), ((50, 400), True), ((24,), False)])
def test_hip_float64_matches_numpy(data, hl, binary):
    """dtype=float64 HIP trainer (f64 MFMA GEMMs, mlp_f64.hip) against the float64 host
    implementation: same loss curve to ~1e-9 relative, same stop epoch, same weights."""
    X, y = data
    if not binary:
        y = (np.arange(len(y)) % 3 + y * 3) % 4     # 4 classes: softmax head
    kw = dict(hidden_layer_sizes=hl, learning_rate_init=0.004, max_iter=60, random_state=42, tol=1e-3)
    a = MLPClassifier(backend="numpy", **kw).fit(X, y)
    b = MLPClassifier(backend="hip", dtype="float64", **kw).fit(X, y)
    assert b._hip_fused            # the two-kernel minibatch step (mlp_fused_f64.hip) ran
    assert b.n_iter_ == a.n_iter_
    np.testing.assert_allclose(b.loss_curve_, a.loss_curve_, rtol=1e-9)
    for u, v in zip(a.coefs_ + a.intercepts_, b.coefs_ + b.intercepts_):
        np.testing.assert_allclose(v, u, rtol=1e-7, atol=1e-9)
    assert (a.predict(X) == b.predict(X)).all()


@pytest.mark.gpu
def test_hip_packed_equals_single(data):
    X, y = data
    lrs = [0.002, 0.005, 0.01]
    packed = [MLPClassifier(hidden_layer_sizes=(32, 64), learning_rate_init=lr, max_iter=12, random_state=42,
                            backend="hip") for lr in lrs]
    fit_packed(packed, X, y)
    single = MLPClassifier(hidden_layer_sizes=(32, 64), learning_rate_init=0.005, max_iter=12, random_state=42,
                           backend="hip").fit(X, y)
    for u, v in zip(single.coefs_, packed[1].coefs_):
        np.testing.assert_allclose(u, v, rtol=1e-6, atol=1e-7)
    assert packed[1].n_iter_ == single.n_iter_


@pytest.mark.gpu
def test_hip_sweep_two_ranks_sharing_the_gpu():
    """The [H] entrypoint with two ranks on one GPU (``--device cuda:0``): its packed jobs run from
    several host threads per rank.  Jobs whose epoch graphs were captured inside those threads saw
    the captures invalidated when another thread's allocations, copies or polling overlapped them
    (two ranks on one GPU made that likely); every job is now built and captured before the threads
    start (``prepare_packed``).  Also: RCCL, which refuses two ranks on one device, is skipped by
    agreement and the averages go through the host."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "hyperparameters_tuning.py",
                        "--device", "cuda:0", "--quiet", "--hidden", "[(16,), (12, 8), (20, 6)]", "--lrs", "0.004",
                        "0.02", "--max-iter", "15"], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Best Global Hyperparameters" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_hip_sweep_concurrent_groups_equal_sequential():
    """run_sweep trains the packed jobs of all hidden configs concurrently (threads + streams):
    results equal the same jobs fitted one after another."""
    from fedmi.hpo.sweep import run_sweep
    from fedmi.models.sklearn_mlp import MLPClassifier, fit_packed
    from fedmi.data.synthetic import make_income_like
    X, y = make_income_like(1200, seed=3)
    hidden, lrs = [(16,), (12, 8), (20, 6)], [0.004, 0.02]
    best, res = run_sweep(X, y, None, hidden, lrs, max_iter=15, backend="hip")
    assert len(res) == 6
    for i, hl in enumerate(hidden):
        ests = [MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=lr, max_iter=15, random_state=42,
                              backend="hip") for lr in lrs]
        fit_packed(ests, X, y)
        for j, e in enumerate(ests):
            r = res[i * len(lrs) + j]
            assert r.hidden == tuple(hl) and r.lr == lrs[j] and r.n_iter == e.n_iter_
            for a, b in zip(r.weights, list(e.coefs_) + list(e.intercepts_)):
                np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("hl", [(50, 400), (400, 200), (12, 8, 6)])
def test_hip_float64_fused_step_equals_layered(data, hl, monkeypatch):
    """The fused float64 minibatch step (2 kernels: row pass + wgrad/Adam, mlp_fused_f64.hip)
    against the layered path (~15 kernels per step, FEDMI_SK_FUSED=0): same epochs, loss curve
    and weights to float64 reordering noise, packed trials included."""
    X, y = data
    lrs = [0.004, 0.02]
    mk = lambda: [MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=lr, max_iter=12, random_state=42,
                                backend="hip", dtype="float64") for lr in lrs]
    fused = fit_packed(mk(), X, y)
    monkeypatch.setenv("FEDMI_SK_FUSED", "0")
    layered = fit_packed(mk(), X, y)
    for f, l in zip(fused, layered):
        assert f._hip_fused and not l._hip_fused
        assert f.n_iter_ == l.n_iter_
        np.testing.assert_allclose(f.loss_curve_, l.loss_curve_, rtol=1e-11)
        for u, v in zip(f.coefs_ + f.intercepts_, l.coefs_ + l.intercepts_):
            np.testing.assert_allclose(u, v, rtol=1e-9, atol=1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("hl,split", [((50, 400), 4), ((50, 200), 4), ((100, 400), 7), ((400, 200), 7),
                                      ((200, 100), 7)])
def test_hip_float64_tile_split_is_bit_identical(data, hl, split, monkeypatch):
    """The tile-split row pass (mlp_fused_f64.hip skf_cs_*: hidden layer 1's forward and input
    gradient cut by output tiles over `split` workgroups per row block, every tile a whole sum with
    the one-workgroup row pass's chunking) gives the one-workgroup row pass's weights bit for bit
    (FEDMI_SK_SPLIT=1), packed trials included; the epoch loss (an atomic sum over row blocks in
    both) to rounding."""
    X, y = data
    lrs = [0.004, 0.02]
    mk = lambda: [MLPClassifier(hidden_layer_sizes=hl, learning_rate_init=lr, max_iter=15, random_state=42,
                                backend="hip", dtype="float64") for lr in lrs]
    monkeypatch.setenv("FEDMI_SK_SPLIT", "1")
    one = fit_packed(mk(), X, y)
    monkeypatch.delenv("FEDMI_SK_SPLIT")
    cut = fit_packed(mk(), X, y)
    for a, b in zip(one, cut):
        assert a._hip_split == 1 and b._hip_split == split, (a._hip_split, b._hip_split)
        assert a.n_iter_ == b.n_iter_
        np.testing.assert_allclose(a.loss_curve_, b.loss_curve_, rtol=1e-13)
        for u, v in zip(a.coefs_ + a.intercepts_, b.coefs_ + b.intercepts_):
            np.testing.assert_array_equal(u, v)


def test_tile_split_rule():
    """The tile-split row pass's slice count (mlp_fused_f64.hip skf_pick_split, host arithmetic):
    at most min(forward tiles, input-gradient tiles, 8) slices, about one workgroup per CU over
    all row blocks and trials, every slice owning a tile of both products; off for other depths
    and wide heads; FEDMI_SK_SPLIT-style overrides."""
    from fedmi.ops import native_available, native
    if not native_available():
        pytest.skip("native extension not built")
    f = native().sk_pick_split
    assert f([14, 50, 400, 1], 1, 200, 0, 256) == 4      # [S]: 4 input-gradient tiles
    assert f([14, 50, 200, 1], 2, 200, 0, 256) == 4
    assert f([14, 100, 400, 1], 2, 200, 0, 256) == 7
    assert f([14, 400, 200, 1], 1, 200, 0, 256) == 7      # 8 would leave the last forward slice empty
    assert f([14, 200, 100, 1], 1, 200, 0, 256) == 7
    assert f([14, 400, 200, 1], 9, 200, 0, 256) == 2      # packed [H] job: 13 row blocks x 9 trials
    assert f([14, 50, 400, 1], 9, 200, 0, 256) == 2
    assert f([14, 50, 400, 1], 1, 200, 0, 32) == 2        # a device with fewer CUs: fewer slices
    assert f([14, 50, 400, 1], 1, 200, 0, 0) == 1         # CU count unknown: no split
    assert f([14, 50, 1], 1, 200, 0, 256) == 1            # one hidden layer
    assert f([14, 50, 400, 5], 1, 200, 0, 256) == 1       # head wider than the narrow path
    assert f([14, 50, 400, 1], 1, 200, 1, 256) == 1       # FEDMI_SK_SPLIT=1: off
    assert f([14, 50, 400, 1], 9, 200, 3, 256) == 2       # asked for 3: the last slice would be empty


@pytest.mark.gpu
def test_hip_sweep_device_predictions_match_the_host_forward(data):
    """The [H] sweep predicts every trial's local rows with float64 products on the GPU
    (fedmi.hpo.sweep._predict_device); its local metrics equal the host forward's
    (MLPClassifier.predict, numpy) on the same weights, trial by trial."""
    from fedmi.fl.metrics import confusion_matrix, metrics_from_confusion
    from fedmi.hpo.sweep import run_sweep
    X, y = data
    best, res = run_sweep(X, y, None, [(50,), (50, 200), (200, 400)], [0.004, 0.02, 0.2], max_iter=12,
                          backend="hip")
    assert len(res) == 9
    for r in res:   # one client: the averaged weights are the local ones
        e = MLPClassifier(hidden_layer_sizes=r.hidden, backend="numpy")
        k = len(r.hidden) + 1
        e.coefs_, e.intercepts_ = r.weights[:k], r.weights[k:]
        e.classes_ = np.unique(y)
        e.n_outputs_, e.out_activation_ = 1, "logistic"
        cm = confusion_matrix(y, e.predict(X), 2)
        assert metrics_from_confusion(cm) == r.local, (r.hidden, r.lr)


@pytest.mark.parametrize("seed,n,epochs,skip", [(42, 8000, 40, 137), (0, 1000, 25, 0), (7, 3, 5, 11)])
def test_native_epoch_orders_are_numpys(seed, n, epochs, skip):
    """The native epoch-order generator (sk_perms.cpp) draws numpy's MT19937 stream bit for bit: the
    same orders as the numpy loop, and the RandomState left in the same state."""
    from fedmi.ops import native_available, native
    if not native_available():
        pytest.skip("native extension not built")
    rs1, rs2 = np.random.RandomState(seed), np.random.RandomState(seed)
    rs1.rand(skip), rs2.rand(skip)                    # e.g. the Glorot init's draws before the orders
    want = np.empty((epochs, n), dtype=np.int32)       # the reference loop (sklearn's shuffle per epoch)
    idx = np.arange(n)
    for e in range(epochs):
        ind = np.arange(n)
        rs1.shuffle(ind)
        idx = idx[ind]
        want[e] = idx
    got = epoch_permutations(rs2, n, epochs)
    np.testing.assert_array_equal(got, want)
    s1, s2 = rs1.get_state(), rs2.get_state()
    np.testing.assert_array_equal(s1[1], s2[1])
    assert s1[2] == s2[2] and rs1.rand() == rs2.rand()
