"""Several clients in one process (fedmi/fl/simulate.py) vs the literal reference client math
(tests/reference_oracle.py: C:63-73 train step, C:75-91 evaluation, C:110-116 FedAvg)."""
import numpy as np
import pytest
import torch

from fedmi.data.sharding import shard_indices
from fedmi.data.tabular import load_tabular
from fedmi.fl.engine import EngineConfig
from fedmi.fl.metrics import confusion_matrix, metric_vector, metrics_from_confusion
from fedmi.fl.simulate import ClientGroup, rounds_to_target
from fedmi.models.mlp import dict_to_flat, init_flat

from .reference_oracle import RefClient, fedavg

DIMS = [14, 50, 200, 2]


def _reference_rounds(X, y, k, rounds, seed):
    idx = [shard_indices(len(X), r, k, mode="compat", seed=seed) for r in range(k)]
    cl = [RefClient(X[i], y[i], DIMS[1:-1], 2, init_flat(DIMS, seed * 1000003 + r)) for r, i in enumerate(idx)]
    glob = []
    for _ in range(rounds):
        ms = []
        for c in cl:
            c.train_one_epoch()
            ms.append(metric_vector(metrics_from_confusion(confusion_matrix(c.y.numpy(), c.predictions(), 2))))
        glob.append(np.mean(ms, axis=0))           # C:169 unweighted mean
        g = fedavg([c.get_weights() for c in cl], [len(i) for i in idx])
        for c in cl:
            c.set_weights(g)
    return dict_to_flat(g, DIMS), np.array(glob)


@pytest.mark.parametrize("k", [1, 3])
def test_torch_client_group_equals_reference(k):
    torch.set_num_threads(1)
    ds = load_tabular()
    X, y = ds.X_train[:3000], ds.y_train[:3000]
    g = ClientGroup(X, y, k, EngineConfig(max_rounds=6, early_stop=False), backend="torch", seed=2)
    g.run(6)
    w, hist = _reference_rounds(X, y, k, 6, seed=2)
    np.testing.assert_allclose(g.global_flat(), w, rtol=0, atol=2e-6)
    np.testing.assert_allclose(g.history()["global"], hist, atol=1e-9)
    assert g.history()["per_rank"].shape == (6, k, 4)


def test_torch_rounds_to_target_keys():
    torch.set_num_threads(1)
    ds = load_tabular()
    out = rounds_to_target(ds.X_train[:2000], ds.y_train[:2000], 2, EngineConfig(max_rounds=40), backend="torch")
    assert set(out) >= {"0.80", "0.83", "early_stop_round", "final_acc", "rounds_run"}
    assert out["rounds_run"] <= 40


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,plain", [("fp32", None), ("bf16", None), ("bf16", False)])
def test_hip_client_group_tracks_torch(dtype, plain):
    """k = 4 HIP clients on one device (classic rounds, device-side sums) vs the torch group.
    bf16: the default (plain-bf16 training forward at world > 1, EngineConfig.plain_fwd None) and
    the split forward (plain_fwd False) both stay within the same drift bound of the fp32 oracle
    (pin the plain forward's drift at N > 1)."""
    ds = load_tabular()
    X, y = ds.X_train, ds.y_train
    cfg = EngineConfig(max_rounds=30, early_stop=False, dtype=dtype, plain_fwd=plain)
    h = ClientGroup(X, y, 4, cfg, backend="hip", seed=1)
    assert all(bool(c.layout["plain_fwd"]) == (dtype == "bf16" and plain is None) for c in h.clients)
    t = ClientGroup(X, y, 4, EngineConfig(max_rounds=30, early_stop=False), backend="torch", seed=1)
    h.run(30)
    t.run(30)
    a, b = h.global_flat(), t.global_flat()
    if dtype == "fp32":
        assert np.abs(a - b).max() / np.abs(b).max() < 1e-4
    else:  # bf16 backward operands: 30 rounds drift a few percent, direction preserved
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 5e-2
    assert h.history()["rounds_run"] == 30
    assert abs(h.history()["global"][-1][0] - t.history()["global"][-1][0]) < (2e-3 if dtype == "fp32" else 1e-2)
