"""Federated hyperparameter sweep with concurrent trials (BASELINE config 5)."""
import os
import subprocess
import sys
from dataclasses import replace

import numpy as np
import pytest
import torch

from fedmi.data.synthetic import make_income_like
from fedmi.fl.engine import EngineConfig, HipRoundEngine, TorchRoundEngine
from fedmi.hpo.fed_sweep import FedTrial, FedTrialGroup, grid, run_fed_sweep
from fedmi.models.mlp import init_flat

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_grid_is_full_product():
    g = grid([(8,), (16, 4)], [0.01, 0.02, 0.03], [1, 2])
    assert len(g) == 12
    assert {(t.hidden, t.lr, t.local_steps) for t in g} == {
        (h, lr, ls) for h in [(8,), (16, 4)] for lr in [0.01, 0.02, 0.03] for ls in [1, 2]}


def test_cpu_group_matches_standalone_engines():
    X, y = make_income_like(600, seed=4)
    trials = grid([(8,), (12, 6)], [0.004, 0.02], [1, 2])
    base = EngineConfig(max_rounds=6, early_stop=False)
    best, done = run_fed_sweep(X, y, 2, None, trials, rounds=6, trials_per_gpu=3, base=base, backend="torch")
    assert len(done) == 8 and all(t.rounds_run == 6 for t in done)
    t = done[5]
    cfg = EngineConfig(hidden=t.hidden, lr=t.lr, local_steps=t.local_steps, max_rounds=6, early_stop=False)
    e = TorchRoundEngine(X, y, 2, cfg, None, init_flat([14, *t.hidden, 2], 0))
    e.run(6)
    np.testing.assert_array_equal(e.history()["global"], t.history["global"])
    assert best.final["accuracy"] == max(x.final["accuracy"] for x in done)


def test_federated_sweep_entrypoint_two_clients_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29633", os.path.join(REPO, "hyperparameters_tuning.py"),
           "--federated", "--device", "cpu", "--rounds", "4", "--hidden", "[(8,)]", "--lrs", "0.004", "0.01",
           "--local-steps", "1", "2", "--trials-per-gpu", "2", "--quiet",
           "--data", os.path.join(REPO, "data", "balanced_income_data.csv")]
    p = subprocess.run(cmd, cwd=REPO, env=dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1"),
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "Best Global Hyperparameters" in p.stdout
    assert "4 trials x 4 rounds" in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("batched", [True, False])
@pytest.mark.parametrize("fused", [True, False])
def test_hip_group_matches_standalone_engines(dtype, batched, fused):
    """Eager group rounds -- trial batches (one launch per kernel for every same-shape trial,
    mixed local steps) or one stream per trial; fused or classic (separate eval kernel)
    evaluation -- give every trial the history of its own engine run alone."""
    X, y = make_income_like(3000, seed=4)
    trials = grid([(50, 200), (16,)], [0.004, 0.01], [1, 2])
    base = EngineConfig(max_rounds=12, early_stop=True, patience=3, tolerance=5e-3, dtype=dtype, graph_rounds=0,
                        fused_eval=fused)
    g = FedTrialGroup(X, y, 2, trials, None, base, backend="hip", batched=batched)
    assert len(g.batches) == (2 if batched else 0)
    g.run(12)
    for t, ge in ((trials[0], g.engines[0]), (trials[5], g.engines[5]), (trials[7], g.engines[7])):
        cfg = replace(base, hidden=t.hidden, lr=t.lr, local_steps=t.local_steps)
        e = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, *t.hidden, 2], 0))
        e.run(12)
        h = e.history()
        assert h["rounds_run"] == t.history["rounds_run"] and h["stop_round"] == t.history["stop_round"]
        np.testing.assert_array_equal(h["global"], t.history["global"])
        np.testing.assert_array_equal(e.global_flat(), ge.global_flat())


def test_reference_h_client_api_runs_grid_and_returns_best():
    """[H] client class (hyperparameters_tuning.py): reference method names, packed grid."""
    sys.path.insert(0, REPO)
    import hyperparameters_tuning as H
    X, y = make_income_like(400, seed=9)
    c = H.FederatedMLPLearning(X, y, 0, 1, backend="numpy")
    assert len(c.X_local) == 400
    params, metrics, weights = c.train_and_evaluate(None, hidden_grid=[(6,), (8, 4)], lr_grid=[0.01, 0.05],
                                                    max_iter=15)
    assert len(c.results) == 4
    best = max(c.results, key=lambda r: r.global_["accuracy"])
    assert params == {"hidden_layer_sizes": best.hidden, "learning_rate": best.lr}
    assert metrics == best.global_ and 0.0 <= metrics["accuracy"] <= 1.0
    assert [w.shape for w in weights] == [w.shape for w in best.weights]
    # single client: the uniform FedAvg is the identity and the confusion matrix is local
    assert c._compute_metrics(y[:10], y[:10])["accuracy"] == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("batched", [True, False])
def test_group_graph_equals_standalone_engines(dtype, batched):
    """One client: the packed group (K trials' rounds captured into one graph, fused
    evaluation) gives every trial bit-identical weights and history to its own engine run
    alone; early stopping inside the group is per trial."""
    X, y = make_income_like(1500, seed=6)
    trials = grid([(16,), (24, 8)], [0.004, 0.02], [1, 2])
    base = EngineConfig(max_rounds=64, patience=3, tolerance=3e-3, dtype=dtype, graph_rounds=8)
    from fedmi.hpo.fed_sweep import FedTrialGroup
    g = FedTrialGroup(X, y, 2, trials, None, base, group_graph_rounds=8, batched=batched)
    g.run(3)     # eager rounds first, then graph replays from an odd start
    g.run(41)
    g.run(16)    # replays only, behind the previous call's history read-back
    assert g.graph is not None
    for t, e in zip(g.trials, g.engines):
        cfg = replace(base, hidden=t.hidden, lr=t.lr, local_steps=t.local_steps)
        ref = HipRoundEngine(X, y, 2, cfg, None, init_flat([14, *t.hidden, 2], 0))
        ref.run(60)
        np.testing.assert_array_equal(ref.global_flat(), e.global_flat())
        h = ref.history()
        assert h["rounds_run"] == t.rounds_run and h["stop_round"] == t.history["stop_round"]
        np.testing.assert_array_equal(h["global"], t.history["global"])


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [True, False])
def test_group_replays_after_history_readback(batched):
    """A run() of graph replays only, behind a run() that read the histories back: the last
    round's metrics are still scored (each engine's round bookkeeping is restored to the state
    the captured rounds leave)."""
    X, y = make_income_like(2000, seed=3)
    trials = grid([(16,), (24, 8)], [0.004], [1, 2])
    base = EngineConfig(max_rounds=40, early_stop=False, dtype="bf16", graph_rounds=8)
    g = FedTrialGroup(X, y, 2, trials, None, base, group_graph_rounds=8, batched=batched)
    g.run(16)
    g.run(16)
    for t, e in zip(g.trials, g.engines):
        ref = HipRoundEngine(X, y, 2, replace(base, hidden=t.hidden, lr=t.lr, local_steps=t.local_steps), None,
                             init_flat([14, *t.hidden, 2], 0))
        ref.run(32)
        np.testing.assert_array_equal(ref.history()["global"], t.history["global"])
        assert t.final["accuracy"] > 0.5


@pytest.mark.gpu
def test_trial_batch_rejects_incompatible_engines():
    """A native trial batch takes engines of one shape, ordered by local steps (descending)."""
    from fedmi.ops import native
    X, y = make_income_like(600, seed=2)
    mk = lambda h, ls: HipRoundEngine(X, y, 2, EngineConfig(hidden=h, local_steps=ls, max_rounds=4, dtype="bf16",
                                                            graph_rounds=0), None, init_flat([14, *h, 2], 0))
    m = native()
    with pytest.raises(RuntimeError, match="shape"):
        m.TrialBatch([mk((16,), 1).engine, mk((24,), 1).engine])
    with pytest.raises(RuntimeError, match="descending"):
        m.TrialBatch([mk((16,), 1).engine, mk((16,), 2).engine])
    tb = m.TrialBatch([mk((16,), 2).engine, mk((16,), 1).engine])
    assert tb.size == 2
