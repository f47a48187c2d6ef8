"""BASELINE config 1: multi-client FedAvg on CPU over gloo (world_size 2 and 3)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, rounds, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.set_num_threads(1)
    from fedmi.data.tabular import load_tabular
    from fedmi.fl.engine import EngineConfig
    from fedmi.fl.trainer import FederatedMLPLearning
    from fedmi.models.mlp import dict_to_flat
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="gloo", device="cpu")
    ds = load_tabular()
    cfg = EngineConfig(max_rounds=rounds)
    tr = FederatedMLPLearning(ds.X_train, ds.y_train, comm.rank, comm.size, comm=comm, config=cfg,
                              mode="correct", backend="torch")
    # one round step by step (reference API) ...
    tr.train_one_epoch()
    local_after = dict_to_flat(tr.get_weights(), tr.engine.dims)
    m = tr.evaluate_local()
    tr.federated_averaging(comm)
    g1 = tr.engine.global_flat()
    # ... then the fused loop
    gm = tr.train_and_evaluate(comm, rounds=rounds - 1, verbose=False)
    test = tr.evaluate_global(ds.X_test, ds.y_test, comm)
    q.put((rank, len(tr.X_local), local_after, m, g1, tr.engine.global_flat(), gm, test,
           tr.history()["per_rank"]))
    comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_fedavg_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 6, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [r[1] for r in res]
    assert sum(sizes) == 8000                       # disjoint IID shards ('correct' mode)
    # round-1 global = sample-size-weighted mean of the post-step local weights (C:110-116)
    expect = sum(r[2] * (n / sum(sizes)) for r, n in zip(res, sizes))
    for r in res:
        np.testing.assert_allclose(r[4], expect, rtol=1e-5, atol=1e-6)
    # all ranks end with bit-identical global weights and identical metric histories
    for r in res[1:]:
        np.testing.assert_array_equal(r[5], res[0][5])
        assert r[6] == res[0][6]
        assert r[7] == res[0][7]
    # global metrics are the unweighted mean of per-rank local metrics (C:169, Q3)
    per_rank = res[0][8]
    np.testing.assert_allclose(np.array(res[0][6]["accuracy"]), per_rank[:, :, 0].mean(axis=1), atol=1e-12)
    # the per-rank metrics of round 1 match each rank's own evaluate_local()
    for k, r in enumerate(res):
        assert abs(per_rank[0, k, 0] - r[3]["accuracy"]) < 1e-12
    assert res[0][7]["accuracy"] > 0.6


def _sampling_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.set_num_threads(1)
    from fedmi.data.tabular import load_tabular
    from fedmi.fl.engine import EngineConfig, TorchRoundEngine
    from fedmi.models.mlp import init_flat
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="gloo", device="cpu")
    ds = load_tabular()
    idx = np.array_split(np.arange(len(ds.y_train)), world)[rank][: 500 + 300 * rank]  # unequal shards
    cfg = EngineConfig(max_rounds=4, early_stop=False, participation=0.5, seed=3)
    e = TorchRoundEngine(ds.X_train[idx], ds.y_train[idx], 2, cfg, comm, init_flat([14, 50, 200, 2], seed=0))
    out = []
    for r in range(3):
        g0 = e.global_flat()
        e.step_train()
        local = e.local_flat()
        e.step_eval()
        e.step_aggregate()
        out.append((list(e.participants(r)), g0, local, e.global_flat(), e._loss))
    q.put((rank, len(idx), out, e.history()))
    comm.close()


def test_partial_participation_over_gloo():
    """Client sampling (participation 0.5 of 4 clients): every rank draws the same 2 clients per
    round, only they train, and the new global is their n_i-weighted mean."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sampling_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [r[1] for r in res]
    for r in range(3):
        parts = res[0][2][r][0]
        assert len(parts) == 2 and all(x[2][r][0] == parts for x in res)
        for k in range(world):
            if k not in parts:   # skipped the local step
                np.testing.assert_array_equal(res[k][2][r][2], res[k][2][r][1])
        n = sum(sizes[k] for k in parts)
        expect = sum(res[k][2][r][2] * (sizes[k] / n) for k in parts)
        for x in res:
            np.testing.assert_allclose(x[2][r][3], expect, rtol=1e-5, atol=1e-6)
            np.testing.assert_array_equal(x[2][r][3], res[0][2][r][3])
    # different rounds draw different sets (seeded per round)
    assert len({tuple(res[0][2][r][0]) for r in range(3)}) > 1
    # global loss and metrics are the sampled clients' (unsampled ones post no loss and score the
    # global model they hold, kept in the per-client history)
    h = res[0][3]
    for r in range(3):
        parts = res[0][2][r][0]
        assert abs(h["loss"][r] - np.mean([res[k][2][r][4] for k in parts])) < 1e-6
        np.testing.assert_allclose(h["global"][r], h["per_rank"][r][parts].mean(axis=0), atol=1e-12)


def _scaled_worker(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch
    torch.set_num_threads(1)
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="gloo", device="cpu")
    a = torch.full((7,), float(rank + 1))
    b = torch.full((5,), float(rank + 1), dtype=torch.bfloat16)
    comm.allreduce_(a, scale=0.25 * (rank + 1))          # sum of w_i * x_i
    comm.allreduce_(b, scale=0.5)
    q.put((rank, a.tolist(), b.float().tolist()))
    comm.close()


def test_comm_scaled_allreduce_over_gloo():
    """Comm.allreduce_(t, scale): the sum of scale_i * t_i (FedAvg weights), fp32 and bf16."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scaled_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=60) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    for _, a, b in out:
        assert a == [0.25 * 1 + 0.5 * 2] * 7
        assert b == [0.5 * 1 + 0.5 * 2] * 5


def _avg_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.set_num_threads(1)
    from fedmi.fl.sklearn_fed import average_estimator_weights, average_many_estimator_weights
    from fedmi.models.sklearn_mlp import MLPClassifier
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="gloo", device="cpu")
    rng = np.random.RandomState(rank)
    ests = []
    for hl in [(3,), (4, 5), (6,)]:
        e = MLPClassifier(hidden_layer_sizes=hl, backend="numpy")
        dims = [2, *hl, 1]
        e.coefs_ = [rng.randn(a, b) for a, b in zip(dims[:-1], dims[1:])]
        e.intercepts_ = [rng.randn(b) for b in dims[1:]]
        ests.append(e)
    many = average_many_estimator_weights(ests, comm)
    one = [average_estimator_weights(e, comm, weighting="uniform") for e in ests]
    q.put((rank, many, one))
    comm.close()


def test_batched_estimator_averaging_matches_one_by_one():
    """The [H] sweep averages all its trials in ONE all-reduce (average_many_estimator_weights):
    the per-trial averages (average_estimator_weights) at world 3 over gloo -- to the last bits, as
    gloo's own reduction order depends on the buffer's length; every rank holds the same result."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, many, one in res:
        assert len(many) == len(one) == 3
        for m_ws, o_ws in zip(many, one):
            assert [w.shape for w in m_ws] == [w.shape for w in o_ws]
            for a, b in zip(m_ws, o_ws):
                np.testing.assert_allclose(a, b, rtol=1e-14, atol=1e-15)
    for _, many, _ in res[1:]:          # every rank holds the same averages
        for a_ws, b_ws in zip(many, res[0][1]):
            for a, b in zip(a_ws, b_ws):
                np.testing.assert_array_equal(a, b)
