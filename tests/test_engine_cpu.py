"""TorchRoundEngine (CPU path) vs a literal transcription of the reference [C] client."""
import numpy as np
import pytest
import torch

from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig, TorchRoundEngine
from fedmi.fl.metrics import confusion_matrix, metrics_from_confusion
from fedmi.models.mlp import (MLPModel, dense_to_image, dict_to_flat, flat_to_dict, image_layout,
                              image_to_dense, init_flat, param_count, param_layout)

from .reference_oracle import RefClient, fedavg


def test_param_layout_matches_reference_named_parameters():
    from .reference_oracle import RefMLP
    dims = [14, 50, 200, 2]
    ref = RefMLP(14, [50, 200], 2)
    names = [(n, tuple(p.shape)) for n, p in ref.named_parameters()]
    assert names == [(n, s) for n, s, _ in param_layout(dims)]
    assert param_count(dims) == 11352 == sum(p.numel() for p in ref.parameters())
    m = MLPModel(14, [50, 200], 2)
    assert [n for n, _ in m.named_parameters()] == [n for n, _ in names]
    # params are views of the flat buffer
    m.flat.zero_()
    assert all(float(p.abs().sum()) == 0 for p in m.parameters())


@pytest.mark.parametrize("dims", [[14, 50, 200, 2], [14, 7, 3], [5, 33, 17, 9, 4]])
def test_image_roundtrip(dims):
    f = init_flat(dims, 3)
    img = dense_to_image(f, dims)
    assert img.size == image_layout(dims)[2] and img.size % 4 == 0
    np.testing.assert_array_equal(image_to_dense(img, dims), f)
    assert abs(img.sum() - f.sum()) < 1e-3   # padding is zero


@pytest.mark.parametrize("dims", [[14, 50, 200, 2], [5, 33, 17, 9, 4]])
def test_image_chunk_swizzle(dims):
    """W_l[n][k] sits at column k ^ swz(n) of image row n, swz(n) = 4 for n mod 16 in [4, 12)
    (fl_common.h fl_swz: the fp32 kernels' bank-conflict-free LDS layout); the 4-float chunks of
    a swizzled row trade places in pairs inside each 16-column block, and the pad columns
    [roundup16(K), ldw) stay zero."""
    f = init_flat(dims, 4)
    img = dense_to_image(f, dims)
    iw, _, _ = image_layout(dims)
    for l, (_, (N, K), off) in enumerate(param_layout(dims)[0::2]):
        W = f[off:off + N * K].reshape(N, K)
        ldw = ((K + 15) & ~15) + 4
        rows = img[iw[l]:iw[l] + ((N + 15) & ~15) * ldw].reshape(-1, ldw)
        for n in range(N):
            sw = 4 if 4 <= n % 16 < 12 else 0
            for k in range(K):
                assert rows[n, k ^ sw] == W[n, k]
            assert not rows[n, (K + 15) & ~15:].any()


def test_dict_flat_roundtrip():
    dims = [14, 50, 200, 2]
    f = init_flat(dims, 1)
    np.testing.assert_array_equal(dict_to_flat(flat_to_dict(f, dims), dims), f)


def test_single_client_rounds_match_reference():
    X, y = make_income_like(600, seed=2)
    dims = [14, 50, 200, 2]
    flat = init_flat(dims, 0)
    cfg = EngineConfig(max_rounds=40, early_stop=False)
    eng = TorchRoundEngine(X, y, 2, cfg, None, flat)
    ref = RefClient(X, y, [50, 200], 2, flat)
    for r in range(40):
        eng.run(1)
        ref.train_one_epoch()
        cm = confusion_matrix(y, ref.predictions(), 2)
        np.testing.assert_allclose(eng.hist.glob[r], list(metrics_from_confusion(cm).values()), atol=1e-12)
    np.testing.assert_allclose(eng.global_flat(), dict_to_flat(ref.get_weights(), dims), rtol=1e-5, atol=1e-6)


def test_fedavg_arithmetic_matches_reference_formula():
    dims = [14, 8, 2]
    rng = np.random.RandomState(0)
    ws = [flat_to_dict(rng.randn(param_count(dims)).astype(np.float32), dims) for _ in range(3)]
    sizes = [100, 250, 57]
    ref = dict_to_flat(fedavg(ws, sizes), dims)
    ours = sum(dict_to_flat(w, dims) * (n / sum(sizes)) for w, n in zip(ws, sizes))
    np.testing.assert_allclose(ours, ref, rtol=1e-6, atol=1e-7)


def test_early_stop_and_lr_schedule_on_real_data():
    from fedmi.data.tabular import load_tabular
    ds = load_tabular()
    dims = [14, 50, 200, 2]
    eng = TorchRoundEngine(ds.X_train, ds.y_train, 2, EngineConfig(max_rounds=300), None, init_flat(dims, 0))
    eng.run(300)
    h = eng.history()
    assert 120 < h["rounds_run"] < 300 and h["stop_round"] == h["rounds_run"]
    acc = h["global"][:, 0]
    assert acc[-1] > 0.82
    # StepLR(30, 0.5) stepped per round (C:46, C:73)
    assert abs(eng.optimizer.param_groups[0]["lr"] - 0.004 * 0.5 ** (h["rounds_run"] // 30)) < 1e-12


def test_fedprox_local_steps_changes_trajectory():
    X, y = make_income_like(300, seed=4)
    dims = [14, 16, 2]
    a = TorchRoundEngine(X, y, 2, EngineConfig(hidden=(16,), local_steps=3, max_rounds=5, early_stop=False),
                         None, init_flat(dims, 0))
    b = TorchRoundEngine(X, y, 2, EngineConfig(hidden=(16,), local_steps=3, prox_mu=0.5, max_rounds=5,
                                               early_stop=False), None, init_flat(dims, 0))
    a.run(5); b.run(5)
    assert not np.allclose(a.global_flat(), b.global_flat())


@pytest.mark.parametrize("backend", ["torch", pytest.param("hip", marks=pytest.mark.gpu)])
def test_train_and_evaluate_early_stop_arguments_take_effect(backend):
    """train_and_evaluate(termination_patience=..., tolerance=...) (C:122) reaches the stop rule
    the engine runs, not only the printed message: the stop round is the host rule's with
    the passed patience."""
    from fedmi.fl.early_stop import EarlyStopper
    from fedmi.fl.trainer import FederatedMLPLearning
    torch.set_num_threads(1)
    X, y = make_income_like(1200, seed=4)
    tr = FederatedMLPLearning(X, y, 0, 1, config=EngineConfig(max_rounds=120), backend=backend, seed=3)
    tr.train_and_evaluate(rounds=120, termination_patience=3, tolerance=5e-3, verbose=False)
    h = tr.history()
    es = EarlyStopper(3, 5e-3)
    stop = next(r + 1 for r, v in enumerate(h["global"]) if es.update(v))
    assert h["stop_round"] == stop == h["rounds_run"]
    with pytest.raises(RuntimeError):
        tr.train_and_evaluate(rounds=130, termination_patience=4, verbose=False)


def test_grad_slab_selection_rule():
    """EngineConfig.grad_slab: 'auto' chooses fp16 gradient partials for the bf16 kernels only
    while every |feature| <= FP16_SLAB_MAX_ABS_X; fp32 kernels never; bad values are refused."""
    from types import SimpleNamespace
    from fedmi.fl.engine import FP16_SLAB_MAX_ABS_X, HipRoundEngine
    pick = HipRoundEngine._pick_slab_f16
    small = SimpleNamespace(X=torch.full((4, 3), FP16_SLAB_MAX_ABS_X))
    big = SimpleNamespace(X=torch.full((4, 3), -2 * FP16_SLAB_MAX_ABS_X))
    assert pick(small, EngineConfig(dtype="bf16"))
    assert not pick(big, EngineConfig(dtype="bf16"))
    assert pick(big, EngineConfig(dtype="bf16", grad_slab="fp16"))
    assert not pick(small, EngineConfig(dtype="bf16", grad_slab="fp32"))
    assert not pick(small, EngineConfig(dtype="fp32", grad_slab="fp16"))
    with pytest.raises(ValueError):
        pick(small, EngineConfig(dtype="bf16", grad_slab="bf16"))


@pytest.mark.parametrize("backend,dtype", [("torch", "fp32"), pytest.param("hip", "fp32", marks=pytest.mark.gpu),
                                           pytest.param("hip", "bf16", marks=pytest.mark.gpu)])
def test_console_streams_rounds_as_they_complete(backend, dtype, capsys):
    """train_and_evaluate(verbose=True) prints each round's reference lines
    (C:139-179) while at most one chunk of <= 16 rounds runs behind them -- not after a 64-round
    chunk -- and the printed text equals the non-streamed print of the same history."""
    import fedmi.obs.console as console
    from fedmi.fl.trainer import FederatedMLPLearning
    torch.set_num_threads(1)
    X, y = make_income_like(1500, seed=8)
    tr = FederatedMLPLearning(X, y, 0, 1, config=EngineConfig(max_rounds=150, dtype=dtype), backend=backend, seed=2)
    seen = []
    real = console.print_history

    def spy(h, patience, start=0, **kw):
        seen.append((start, h["rounds_run"], tr.engine.rounds_issued))
        return real(h, patience, start=start, **kw)
    import fedmi.fl.trainer as trainer_mod
    old = trainer_mod.print_history
    trainer_mod.print_history = spy
    try:
        tr.train_and_evaluate(rounds=150, termination_patience=3, tolerance=5e-3, verbose=True)
    finally:
        trainer_mod.print_history = old
    out = capsys.readouterr().out
    h = tr.history()
    assert h["stop_round"] > 0
    printed_upto = 0
    for start, upto, issued in seen:
        assert start == printed_upto
        # rounds issued beyond the last printed round: at most one chunk in flight
        if upto < h["rounds_run"]:
            assert issued - upto <= 16, (issued, upto)
        printed_upto = upto
    assert printed_upto == h["rounds_run"]
    assert len([s for s in seen if s[1] > s[0]]) >= h["rounds_run"] // 16   # printed chunk by chunk
    lines = []
    real(h, 3, print_fn=lambda s, **k: lines.append(s))
    assert out == "".join(s + "\n" for s in lines)
