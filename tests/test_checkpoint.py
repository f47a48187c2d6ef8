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
    assert sorted(os.listdir(tmp_path)) == ["client0.safetensors", "meta.json", "weights.safetensors"]
    ck = load_checkpoint(str(tmp_path), rank=0)
    model = MLPModel(14, [50, 200], 2)
    # plain torch load of the reference key names: model.{0,2,4}.{weight,bias}
    sd = {k: torch.as_tensor(v) for k, v in ck["weights"].items()}
    ref = torch.nn.Sequential(torch.nn.Linear(14, 50), torch.nn.ReLU(), torch.nn.Linear(50, 200), torch.nn.ReLU(),
                              torch.nn.Linear(200, 2))
    ref.load_state_dict({k.split("model.", 1)[1]: v for k, v in sd.items()})
    assert set(ck["weights"]) == {n for n, _ in model.named_parameters()}
    meta = json.load(open(tmp_path / "meta.json"))
    assert meta["rounds"] == 2 and meta["dims"] == dims


def test_resume_rejects_mismatched_dims(tmp_path):
    X, y = make_income_like(200, seed=1)
    e = _engine(X, y, [14, 8, 2])
    e.run(1)
    save_checkpoint(str(tmp_path), e)
    with pytest.raises(ValueError):
        resume(str(tmp_path), _engine(X, y, [14, 9, 2]))
