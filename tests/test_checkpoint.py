"""Checkpoint / resume: a resumed run continues bit-identically."""
import json
import os

import numpy as np
import pytest
import torch

from fedmi.ckpt.checkpoint import load_checkpoint, resume, save_checkpoint
from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig, TorchRoundEngine
from fedmi.models.mlp import MLPModel, init_flat


def _engine(X, y, dims, **kw):
    cfg = EngineConfig(hidden=tuple(dims[1:-1]), max_rounds=60, patience=3, tolerance=2e-3, **kw)
    return TorchRoundEngine(X, y, dims[-1], cfg, None, init_flat(dims, 4))


@pytest.mark.parametrize("split", [5, 31])
def test_torch_resume_is_exact(tmp_path, split):
    X, y = make_income_like(700, seed=3)
    dims = [14, 24, 16, 2]
    # step_size 30: split=31 resumes after the first StepLR decay
    full = _engine(X, y, dims)
    full.run(40)
    a = _engine(X, y, dims)
    a.run(split)
    save_checkpoint(str(tmp_path), a)
    b = _engine(X, y, dims)
    assert resume(str(tmp_path), b) == split
    assert b.optimizer.param_groups[0]["lr"] == a.optimizer.param_groups[0]["lr"]
    b.run(40 - split)
    ha, hb = full.history(), b.history()
    assert ha["rounds_run"] == hb["rounds_run"]
    np.testing.assert_array_equal(ha["global"], hb["global"])
    assert ha["stop_round"] == hb["stop_round"]
    np.testing.assert_array_equal(full.global_flat(), b.global_flat())


def test_checkpoint_layout_is_reference_state_dict(tmp_path):
    X, y = make_income_like(300, seed=1)
    dims = [14, 50, 200, 2]
    e = _engine(X, y, dims)
    e.run(2)
    save_checkpoint(str(tmp_path), e)
    assert sorted(os.listdir(tmp_path)) == ["client0.r2.safetensors", "meta.json", "weights.r2.safetensors",
                                            "weights.safetensors"]
    e.run(1)
    save_checkpoint(str(tmp_path), e)   # the next round's set replaces (prunes) round 2's
    assert sorted(os.listdir(tmp_path)) == ["client0.r3.safetensors", "meta.json", "weights.r3.safetensors",
                                            "weights.safetensors"]
    ck = load_checkpoint(str(tmp_path), rank=0)
    model = MLPModel(14, [50, 200], 2)
    # plain torch load of the reference key names: model.{0,2,4}.{weight,bias}
    sd = {k: torch.as_tensor(v) for k, v in ck["weights"].items()}
    ref = torch.nn.Sequential(torch.nn.Linear(14, 50), torch.nn.ReLU(), torch.nn.Linear(50, 200), torch.nn.ReLU(),
                              torch.nn.Linear(200, 2))
    ref.load_state_dict({k.split("model.", 1)[1]: v for k, v in sd.items()})
    assert set(ck["weights"]) == {n for n, _ in model.named_parameters()}
    meta = json.load(open(tmp_path / "meta.json"))
    assert meta["rounds"] == 3 and meta["dims"] == dims


def test_checkpoint_crash_before_meta_keeps_previous_round(tmp_path, monkeypatch):
    """A crash after the new round's weight files are in place but before meta.json is rewritten
    leaves the previous round's complete set loadable; a file from another round under
    meta.json's name is refused."""
    import fedmi.ckpt.checkpoint as ck
    X, y = make_income_like(300, seed=1)
    dims = [14, 8, 2]
    e = _engine(X, y, dims)
    e.run(2)
    save_checkpoint(str(tmp_path), e)
    g2 = e.global_flat()
    e.run(1)

    def crash(*a, **k):
        raise RuntimeError("simulated crash before meta.json")
    monkeypatch.setattr(ck, "_publish_meta", crash)
    with pytest.raises(RuntimeError):
        save_checkpoint(str(tmp_path), e)
    monkeypatch.undo()
    assert {"client0.r3.safetensors", "weights.r3.safetensors"} <= set(os.listdir(tmp_path))
    b = _engine(X, y, dims)
    assert resume(str(tmp_path), b) == 2
    np.testing.assert_array_equal(b.global_flat(), g2)
    # a round-3 file under round 2's name: the header round check refuses it
    os.replace(tmp_path / "client0.r3.safetensors", tmp_path / "client0.r2.safetensors")
    with pytest.raises(ValueError, match="round"):
        resume(str(tmp_path), _engine(X, y, dims))


def test_sklearn_run_crash_before_meta_keeps_previous_round(tmp_path, monkeypatch):
    import fedmi.ckpt.checkpoint as ck
    rs = np.random.RandomState(0)
    mk = lambda: [rs.randn(4, 3), rs.randn(3, 1), rs.randn(3), rs.randn(1)]
    w1l, w1g = mk(), mk()
    ck.save_sklearn_run(str(tmp_path), 0, 1, w1g, w1l, {"history": []})
    monkeypatch.setattr(ck, "_publish_meta", lambda *a, **k: (_ for _ in ()).throw(RuntimeError("crash")))
    with pytest.raises(RuntimeError):
        ck.save_sklearn_run(str(tmp_path), 0, 2, mk(), mk(), {"history": []})
    monkeypatch.undo()
    out = ck.load_sklearn_run(str(tmp_path), 0)
    assert out["meta"]["rounds"] == 1
    for a, b in zip(out["local"] + out["global"], w1l + w1g):
        np.testing.assert_array_equal(a, b)
    ck.save_sklearn_run(str(tmp_path), 0, 2, w1g, w1l, {"history": []})
    assert sorted(os.listdir(tmp_path)) == ["client0.r2.safetensors", "global.r2.safetensors", "meta.json"]


def test_resume_rejects_mismatched_dims(tmp_path):
    X, y = make_income_like(200, seed=1)
    e = _engine(X, y, [14, 8, 2])
    e.run(1)
    save_checkpoint(str(tmp_path), e)
    with pytest.raises(ValueError):
        resume(str(tmp_path), _engine(X, y, [14, 9, 2]))


def test_sklearn_layout_roundtrip(tmp_path):
    """[S]/[H] exchange layout (S:26): coefs_ [in, out] then intercepts_, float64."""
    from fedmi.ckpt.checkpoint import load_sklearn_weights, save_sklearn_weights, sklearn_to_torch_layout
    rs = np.random.RandomState(0)
    dims = [14, 50, 400, 1]
    coefs = [rs.randn(a, b) for a, b in zip(dims[:-1], dims[1:])]
    inter = [rs.randn(b) for b in dims[1:]]
    save_sklearn_weights(str(tmp_path / "w.safetensors"), coefs + inter)
    back = load_sklearn_weights(str(tmp_path / "w.safetensors"))
    assert len(back) == 6 and all(b.dtype == np.float64 for b in back)
    for a, b in zip(coefs + inter, back):
        np.testing.assert_array_equal(a, b)
    t = sklearn_to_torch_layout(back)
    assert t["model.2.weight"].shape == (400, 50) and t["model.4.bias"].shape == (1,)
    with pytest.raises(ValueError):
        save_sklearn_weights(str(tmp_path / "bad.safetensors"), coefs)   # intercepts missing


def test_sklearn_flow_save_resume_exact(tmp_path):
    """[S] rounds with --save, interrupted after round 2 and resumed: same global weights and
    history as the uninterrupted run (warm start, numpy float64 backend)."""
    import importlib
    S = importlib.import_module("FL_SkLearn_MLPClassifier_Limitation")
    from fedmi.data.tabular import load_tabular
    ds = load_tabular(with_mean=False)
    X, y = ds.X_train[:600], ds.y_train[:600]
    mk = lambda: S.FederatedMLPLearning(X, y, 0, 1, hidden=(8, 6), max_iter=15, warm_start=True, backend="numpy")
    full = mk()
    h_full = full.train_and_evaluate(None, rounds=4)
    a = mk()
    a.train_and_evaluate(None, rounds=2, save=str(tmp_path))
    b = mk()
    h_b = b.train_and_evaluate(None, rounds=4, resume=str(tmp_path))
    assert [r["global"] for r in h_b] == [r["global"] for r in h_full]
    for u, v in zip(full.global_weights, b.global_weights):
        np.testing.assert_array_equal(u, v)


def test_hpo_sweep_save_resume_reuses_trials(tmp_path):
    from fedmi.data.tabular import load_tabular
    from fedmi.hpo.sweep import load_sweep, run_sweep, save_sweep
    ds = load_tabular(with_mean=False)
    X, y = ds.X_train[:400], ds.y_train[:400]
    best, res = run_sweep(X, y, None, [(5,)], [0.01, 0.02], max_iter=5, backend="numpy")
    save_sweep(str(tmp_path), res, best, {"world": 1})
    done = load_sweep(str(tmp_path))
    calls = []
    best2, res2 = run_sweep(X, y, None, [(5,), (6,)], [0.01, 0.02], max_iter=5, backend="numpy", done=done,
                            on_trial=lambda r: calls.append(r.hidden))
    assert calls == [(6,), (6,)]                 # only the new hidden config trained
    assert [r.global_ for r in res2[:2]] == [r.global_ for r in res]
    for u, v in zip(res2[0].weights, res[0].weights):
        np.testing.assert_array_equal(u, v)
    assert os.path.isfile(tmp_path / "best.safetensors")
    # a checkpoint of another run (different client count) is refused, not mixed in
    with pytest.raises(ValueError, match="world"):
        load_sweep(str(tmp_path), expect={"world": 2})
    assert len(load_sweep(str(tmp_path), expect={"world": 1})) == 2


def test_hpo_sweep_incremental_checkpoint(tmp_path):
    """[H] --save writes after every trial: a sweep interrupted after k trials resumes them."""
    from fedmi.data.tabular import load_tabular
    from fedmi.hpo.sweep import load_sweep, run_sweep, save_sweep
    ds = load_tabular(with_mean=False)
    X, y = ds.X_train[:400], ds.y_train[:400]
    partial = []

    def on_trial(r):
        partial.append(r)
        save_sweep(str(tmp_path), partial, None, {"world": 1})
        if len(partial) == 3:
            raise KeyboardInterrupt  # "crash" after the third trial

    with pytest.raises(KeyboardInterrupt):
        run_sweep(X, y, None, [(5,), (6,)], [0.01, 0.02], max_iter=5, backend="numpy", on_trial=on_trial)
    done = load_sweep(str(tmp_path), expect={"world": 1})
    assert [(r.hidden, r.lr) for r in done] == [((5,), 0.01), ((5,), 0.02), ((6,), 0.01)]


@pytest.mark.gpu
def test_wide_client_checkpoint_exact(tmp_path):
    from fedmi.data.synthetic import make_income_like
    from fedmi.fl.wide import WideClient, load_wide, save_wide
    dev = torch.device("cuda", 0)
    Xn, yn = make_income_like(1024, seed=8)
    X, y = torch.as_tensor(Xn, device=dev), torch.as_tensor(yn, device=dev)
    mk = lambda: WideClient(X, y, [14, 256, 128, 2], micro_batch=512, dtype="bf16", seed=3)
    a = mk()
    for _ in range(2):
        a.run_round()
    save_wide(str(tmp_path), a)
    b = mk()
    assert load_wide(str(tmp_path), b) == 2
    a.run_round()
    b.run_round()
    a.sync(); b.sync()
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)


def test_hpo_sweep_save_overwrites_stale_trial_files(tmp_path):
    """a --save directory left by an earlier run (other data / max_iter) must not lend
    its trial weights to this run's sweep.json: files of another run are rewritten, a mismatched
    file under this run's sweep.json is refused on load, duplicate trials are saved once, and
    nearby learning rates get distinct files."""
    from fedmi.data.tabular import load_tabular
    from fedmi.hpo.sweep import _trial_file, TrialResult, load_sweep, run_sweep, save_sweep
    ds = load_tabular(with_mean=False)
    X, y = ds.X_train[:400], ds.y_train[:400]
    best_a, res_a = run_sweep(X, y, None, [(5,)], [0.01], max_iter=3, backend="numpy")
    save_sweep(str(tmp_path), res_a, best_a, {"world": 1, "max_iter": 3})
    best_b, res_b = run_sweep(X, y, None, [(5,)], [0.01], max_iter=9, backend="numpy")
    save_sweep(str(tmp_path), res_b + res_b, best_b, {"world": 1, "max_iter": 9})
    back = load_sweep(str(tmp_path), expect={"max_iter": 9})
    assert len(back) == 1
    for u, v in zip(back[0].weights, res_b[0].weights):
        np.testing.assert_array_equal(u, v)
    # swap in the other run's file under this run's name: refused
    save_sweep(str(tmp_path / "other"), res_a, best_a, {"world": 1, "max_iter": 3})
    os.replace(tmp_path / "other" / _trial_file(res_a[0]), tmp_path / _trial_file(res_b[0]))
    with pytest.raises(ValueError, match="another run"):
        load_sweep(str(tmp_path))
    mk = lambda lr: TrialResult((5,), lr, {}, {}, 1, [])
    assert _trial_file(mk(0.0012345671)) != _trial_file(mk(0.0012345674))
