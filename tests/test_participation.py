"""Client sampling (partial participation) on both engines, and resume of a sampled run.

Semantics (EngineConfig.participation): each round a seeded draw of max(1, round(f * k))
clients trains and is averaged with weights n_i / (sum of the sampled n_j); the others keep the
global model.  StepLR follows the round index for everyone, Adam's bias correction each client's
own step count; global metrics / loss are the sampled clients'."""
import numpy as np
import pytest
import torch

from fedmi.ckpt.checkpoint import resume, save_checkpoint
from fedmi.data.tabular import load_tabular
from fedmi.fl.engine import EngineConfig
from fedmi.fl.simulate import ClientGroup


def _data(n=2400):
    ds = load_tabular()
    return ds.X_train[:n], ds.y_train[:n]


def _group(backend, rounds=14, **kw):
    X, y = _data()
    cfg = EngineConfig(max_rounds=rounds, participation=0.5, seed=5, patience=3, tolerance=3e-3, **kw)
    return ClientGroup(X, y, 4, cfg, backend=backend, seed=1)


def _resume_case(backend, tmp_path, split):
    full = _group(backend)
    full.run(14)
    a = _group(backend)
    a.run(split)
    for r, e in enumerate(a.clients):
        save_checkpoint(str(tmp_path), e)
    b = _group(backend)
    for e in b.clients:
        assert resume(str(tmp_path), e) == split
    b.rounds = split
    b.run(14 - split)
    return full, b


@pytest.mark.parametrize("split", [4, 9])
def test_torch_sampled_run_resumes_exactly(tmp_path, split):
    """a client that skipped rounds has fewer Adam steps than rounds; the checkpoint
    keeps each client's own step count, so the resumed run equals the uninterrupted one."""
    torch.set_num_threads(1)
    full, b = _resume_case("torch", tmp_path, split)
    for ea, eb in zip(full.clients, b.clients):
        st_a = ea.optimizer.state[next(iter(ea.model.parameters()))]["step"]
        st_b = eb.optimizer.state[next(iter(eb.model.parameters()))]["step"]
        assert float(st_a) == float(st_b) < 14      # sampled: fewer steps than rounds
        np.testing.assert_array_equal(ea.global_flat(), eb.global_flat())
        assert ea.optimizer.param_groups[0]["lr"] == eb.optimizer.param_groups[0]["lr"]
    ha, hb = full.history(), b.history()
    assert ha["rounds_run"] == hb["rounds_run"]
    np.testing.assert_array_equal(ha["global"], hb["global"])
    np.testing.assert_array_equal(ha["loss"], hb["loss"])


@pytest.mark.gpu
def test_hip_sampling_tracks_torch():
    """HIP engines read the per-round device table (weights, sampled set, own-step Adam
    scalars): the sampled run tracks the torch engines' within fp32 rounding."""
    h = _group("hip", rounds=20, early_stop=False)
    t = _group("torch", rounds=20, early_stop=False)
    h.run(20)
    t.run(20)
    a, b = h.global_flat(), t.global_flat()
    # (the torch engine divides by the sampled sum after the all-reduce, the HIP engines pre-scale:
    # last-bit differences that Adam's normalisation amplifies on a few near-zero-gradient weights)
    assert np.linalg.norm(a - b) / np.linalg.norm(b) < 5e-4
    assert np.abs(a - b).max() / np.abs(b).max() < 5e-3
    np.testing.assert_allclose(h.history()["global"], t.history()["global"], atol=3e-3)
    np.testing.assert_allclose(h.history()["loss"], t.history()["loss"], rtol=1e-4)


@pytest.mark.gpu
def test_hip_sampled_run_resumes_exactly(tmp_path):
    full, b = _resume_case("hip", tmp_path, 7)
    np.testing.assert_array_equal(full.global_flat(), b.global_flat())
    ha, hb = full.history(), b.history()
    assert ha["rounds_run"] == hb["rounds_run"]
    np.testing.assert_array_equal(ha["global"], hb["global"])
