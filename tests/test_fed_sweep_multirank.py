"""Packed federated sweep (BASELINE config 5) with several clients: two ranks sharing ``cuda:0``
(the 1-GPU box), FedAvg of all trials as one host (gloo) all-reduce per round.  Every trial of
the group -- native trial batches (classic rounds: pack, train, Adam, eval and finalize kernels
each launched once per batch) or one stream per trial -- must end with the weights and history
of the same trial run alone as an ordinary two-client engine."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2
ROUNDS = 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        from dataclasses import replace

        from fedmi.data.synthetic import make_income_like
        from fedmi.fl.engine import EngineConfig, HipRoundEngine
        from fedmi.hpo.fed_sweep import FedTrialGroup, grid
        from fedmi.models.mlp import init_flat
        from fedmi.parallel.comm import Comm
        comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
        comm.peer_allreduce = False
        X, y = make_income_like(1800 + 200 * rank, seed=30 + rank)
        trials = grid([(24, 8), (16,)], [0.004, 0.01], [1, 2])
        base = EngineConfig(max_rounds=ROUNDS, patience=3, tolerance=3e-3, dtype="bf16", graph_rounds=0)
        res = {}
        for batched in (True, False):
            g = FedTrialGroup(X, y, 2, trials, comm, base, batched=batched)
            assert len(g.batches) == (2 if batched else 0)
            g.run(4)
            g.run(ROUNDS - 4)
            res[batched] = [(e.global_flat(), t.history) for t, e in zip(g.trials, g.engines)]
        alone = []
        for t in trials:
            cfg = replace(base, hidden=t.hidden, lr=t.lr, local_steps=t.local_steps)
            e = HipRoundEngine(X, y, 2, cfg, comm, init_flat([14, *t.hidden, 2], rank))
            assert e.aggregation == "host", e.aggregation
            e.run(ROUNDS)
            alone.append((e.global_flat(), e.history()))
        res["alone"] = alone
        comm.Barrier()
        q.put((rank, res, None))
        comm.close()
    except Exception:  # noqa: BLE001 -- reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_group_two_ranks_matches_standalone_engines():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=110) for _ in range(WORLD)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, res, err in out:
        assert err is None, f"rank {rank}:\n{err}"
        for batched in (True, False):
            for i, ((w, h), (wa, ha)) in enumerate(zip(res[batched], res["alone"])):
                msg = f"rank {rank} trial {i} batched={batched}"
                np.testing.assert_array_equal(w, wa, err_msg=msg)
                assert h["rounds_run"] == ha["rounds_run"] and h["stop_round"] == ha["stop_round"], msg
                np.testing.assert_array_equal(h["global"], ha["global"], err_msg=msg)
                np.testing.assert_array_equal(h["per_rank"], ha["per_rank"], err_msg=msg)
                np.testing.assert_array_equal(h["loss"], ha["loss"], err_msg=msg)
    # both clients hold the same global model of every trial
    for (w0, _), (w1, _) in zip(out[0][1][True], out[1][1][True]):
        np.testing.assert_array_equal(w0, w1)
    for p in procs:
        assert p.exitcode == 0
