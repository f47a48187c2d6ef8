"""One-shot xGMI peer all-reduce (fedmi/ops/csrc/peer_allreduce.hip, fedmi/parallel/peer.py).

The 1-GPU box cannot exercise real xGMI links, so two ranks share ``cuda:0``: every rank
still maps the other's allocation through HIP IPC and the kernel's publish / wait / pull
protocol runs unchanged (the reads just stay on one device).  Checks:

* the collective set-up + self-test succeeds on every rank (exact payload, both parities);
* the fused round engine aggregating with the peer kernel (fp32, and bf16 with the packed
  LDS-image epilogue that replaces the pack kernel) is bit-identical to the same engine
  aggregating through the host (gloo), for eager rounds, graph-captured rounds and the
  reference step-by-step API.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_engine(comm, peer: bool, dtype: str, X, y, flat, eval_fedavg: bool = True, lagged: bool = True,
                hidden=(50, 200), expect_ll=None):
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    comm.peer_allreduce = peer
    cfg = EngineConfig(hidden=tuple(hidden), max_rounds=30, early_stop=False, dtype=dtype, graph_rounds=4,
                       eval_fedavg=eval_fedavg, lagged_eval=lagged)
    e = HipRoundEngine(X, y, 2, cfg, comm, flat)
    lag = lagged and dtype == "bf16"
    assert e.aggregation == (("xgmi-oneshot+adam" if lag else "xgmi-oneshot") if peer else "host"), e.aggregation
    assert bool(e.engine.lagged) == lag, (e.engine.lagged, lagged, dtype)
    assert bool(e.engine.adam_exchange) == (lag and peer)
    if expect_ll is not None:  # LL weight chunks of the Adam-fused exchange (peer_device.h)
        assert bool(e._peer.uses_ll) == expect_ll
    e.run(3)                       # eager rounds
    cms = []
    for _ in range(2):             # reference step-by-step API
        e.step_train()
        cms.append(e.step_eval())
        e.step_aggregate()
    e.run(9)                       # graph-captured chunks
    e.sync_history()
    return e.global_flat(), e.history(), np.stack(cms)


def _run_early_stop(comm, peer: bool, X, y, flat, lagged: bool = True):
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    comm.peer_allreduce = peer
    cfg = EngineConfig(max_rounds=200, patience=4, tolerance=2e-3, dtype="bf16", graph_rounds=8,
                       lagged_eval=lagged)
    e = HipRoundEngine(X, y, 2, cfg, comm, flat)
    # early stopping runs lagged rounds: with the peer data plane the metrics are exchanged and
    # folded inside the next round's Adam kernel; over an external all-reduce (here gloo) they are
    # folded one round late and a round run past the stop is discarded bit-exactly (late fold)
    assert bool(e.engine.lagged) == lagged
    assert bool(e.engine.late_fold) == (lagged and not peer)
    e.run(200)
    return e.global_flat(), e.history()


def _worker(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        from fedmi.data.synthetic import make_income_like
        from fedmi.models.mlp import init_flat
        from fedmi.parallel.comm import Comm
        from fedmi.parallel.peer import make_peer_allreduce, selftest
        comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
        dev = comm.device
        res = {}
        # raw communicator: odd lengths exercise the scalar tail of the kernel
        for n in (4099, 50003):
            h = make_peer_allreduce(comm, n, dev, timeout_s=30.0)
            res[f"open{n}"] = h is not None
            if h is not None:
                res[f"self{n}"] = bool(all(comm.allgather(selftest(h, comm, dev, calls=6))))
                comm.Barrier()
                h.close()
        X, y = make_income_like(2400, seed=20 + rank)
        flat = init_flat([14, 50, 200, 2], 3)
        for dtype in ("fp32", "bf16"):
            # bf16 default: lagged evaluation (scored in the next train kernel); fp32: fused
            # evaluation + all-reduce kernel
            a = _run_engine(comm, True, dtype, X, y, flat)
            b = _run_engine(comm, False, dtype, X, y, flat, lagged=False)     # host (gloo) aggregation
            c = _run_engine(comm, True, dtype, X, y, flat, False, False)      # separate eval / peer kernels
            d = _run_engine(comm, True, dtype, X, y, flat, True, False)       # fused eval + all-reduce kernel
            res[dtype] = (a, b, c, d)
        # early stop: rounds past the stop (non-live) must reproduce the stop round's model
        res["es"] = (_run_early_stop(comm, True, X, y, flat), _run_early_stop(comm, False, X, y, flat),
                     _run_early_stop(comm, True, X, y, flat, lagged=False))
        torch.cuda.synchronize()
        comm.Barrier()
        q.put((rank, res, None))
        comm.close()
    except Exception:  # noqa: BLE001 -- reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_peer_allreduce_two_ranks_one_gpu():
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
        for n in (4099, 50003):
            assert res[f"open{n}"] and res[f"self{n}"], (rank, n, res)
        for dtype in ("fp32", "bf16"):
            (wa, ha, ca), (wb, hb, cb), (wc, hc, cc), (wd, hd, cd) = res[dtype]
            for name, (w, h) in (("separate kernels", (wc, hc)), ("eval+fedavg kernel", (wd, hd))):
                np.testing.assert_array_equal(w, wb, err_msg=f"{dtype} weights ({name})")
                np.testing.assert_array_equal(h["global"], hb["global"], err_msg=f"{dtype} metrics ({name})")
                np.testing.assert_array_equal(h["loss"], hb["loss"], err_msg=f"{dtype} loss ({name})")
            np.testing.assert_array_equal(wa, wb, err_msg=f"{dtype} weights")
            np.testing.assert_array_equal(ha["global"], hb["global"])
            np.testing.assert_array_equal(ha["per_rank"], hb["per_rank"])
            np.testing.assert_array_equal(ha["loss"], hb["loss"])
            np.testing.assert_array_equal(ca, cb)
            assert ha["rounds_run"] == 14
        (we, he), (wf, hf), (wg, hg) = res["es"]
        assert he["stop_round"] > 0 and he["stop_round"] == hf["stop_round"], (he["stop_round"], hf["stop_round"])
        assert he["rounds_run"] == hf["rounds_run"] == hg["rounds_run"]
        np.testing.assert_array_equal(we, wf)
        np.testing.assert_array_equal(wg, wf)
        np.testing.assert_array_equal(he["global"], hf["global"])
        np.testing.assert_array_equal(he["loss"], hf["loss"])
        np.testing.assert_array_equal(hg["global"], hf["global"])
    # both ranks hold the same global model
    for dtype in ("fp32", "bf16"):
        np.testing.assert_array_equal(out[0][1][dtype][0][0], out[1][1][dtype][0][0])
    for p in procs:
        assert p.exitcode == 0


def _worker4(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        from fedmi.data.synthetic import make_income_like
        from fedmi.models.mlp import init_flat
        from fedmi.parallel.comm import Comm
        from fedmi.parallel.peer import make_peer_allreduce, selftest
        comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
        dev = comm.device
        h = make_peer_allreduce(comm, 3001, dev, timeout_s=30.0, n_chunks=48)
        ok = h is not None and bool(all(comm.allgather(selftest(h, comm, dev, calls=4))))
        comm.Barrier()
        if h is not None:
            h.close()
        X, y = make_income_like(900 + 100 * rank, seed=30 + rank)   # unequal shards: n_i / N weights
        # a small model: the Adam blocks of all four ranks must be resident on the ONE shared GPU
        # at once (each waits for the others' chunks; on separate GPUs that always holds)
        hidden = (24, 12)
        flat = init_flat([14, *hidden, 2], 5)
        a = _run_engine(comm, True, "bf16", X, y, flat, hidden=hidden, expect_ll=True)
        # the same exchange with publish / wait / pull weight chunks (FEDMI_PEER_LL=0)
        os.environ["FEDMI_PEER_LL"] = "0"
        try:
            a0 = _run_engine(comm, True, "bf16", X, y, flat, hidden=hidden, expect_ll=False)
        finally:
            del os.environ["FEDMI_PEER_LL"]
        # ... and by reduce-scatter + all-gather on the LL ring (FEDMI_PEER_RSAG=1)
        os.environ["FEDMI_PEER_RSAG"] = "1"
        try:
            h = make_peer_allreduce(comm, 3001, dev, timeout_s=30.0, n_chunks=48)   # + the RS+AG self-test
            ok = ok and h is not None and bool(h.uses_rsag)
            comm.Barrier()
            if h is not None:
                h.close()
            ar = _run_engine(comm, True, "bf16", X, y, flat, hidden=hidden, expect_ll=True)
        finally:
            del os.environ["FEDMI_PEER_RSAG"]
        # classic rounds over the standalone peer kernel: the same rank-order sums (gloo's
        # 4-rank reduction order differs, so the host path is not a bitwise reference here)
        b = _run_engine(comm, True, "bf16", X, y, flat, True, False, hidden=hidden)
        torch.cuda.synchronize()
        comm.Barrier()
        q.put((rank, (ok, a, b, a0, ar), None))
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [4, 8])
def test_peer_many_ranks_lagged_adam_exchange(world):
    """W = 4 and W = 8 = PEER_MAX_WORLD, the world of an MI355X node (every unrolled rank loop,
    every chunk-flag row and all 8 sources of the LL ring in use): self-tests of all three
    protocols (standalone pull, publish / wait / pull chunks, LL chunks) pass, and the lagged
    engine with FedAvg inside the Adam kernel -- LL weight chunks (value + call index in one
    8-byte push) and publish / wait / pull chunks alike -- equals classic rounds over the
    standalone peer kernel bit for bit, with unequal shard sizes; every rank ends with the same
    global model.  All ranks share cuda:0 (the 1-GPU box), so the pulls stay on one device."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker4, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=110 + 30 * world) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, res, err in out:
        assert err is None, f"rank {rank}:\n{err}"
        ok, (wa, ha, ca), (wb, hb, cb), (w0, h0, c0), (wr, hr, cr) = res
        assert ok
        np.testing.assert_array_equal(wr, wb)
        np.testing.assert_array_equal(hr["global"], hb["global"])
        np.testing.assert_array_equal(cr, cb)
        np.testing.assert_array_equal(wa, wb)
        np.testing.assert_array_equal(w0, wb)
        bad = np.flatnonzero((h0["global"] != hb["global"]).any(axis=1))
        np.testing.assert_array_equal(h0["global"], hb["global"], err_msg=(
            f"rank {rank}: pull-exchange metrics differ at rounds {bad.tolist()}: "
            f"pull {h0['global'][bad].tolist()} classic {hb['global'][bad].tolist()}; per-rank pull "
            f"{np.asarray(h0['per_rank'])[bad].tolist()} classic {np.asarray(hb['per_rank'])[bad].tolist()}"))
        np.testing.assert_array_equal(c0, cb)
        np.testing.assert_array_equal(ha["global"], hb["global"])
        np.testing.assert_array_equal(ha["per_rank"], hb["per_rank"])
        np.testing.assert_array_equal(ca, cb)
    for r in range(1, world):
        np.testing.assert_array_equal(out[0][1][1][0], out[r][1][1][0])


def _run_prod(comm, X, y, flat, n_total, lagged: bool, rounds: int):
    """The bench's N > 1 round at the reference shape: MLP 14-50-200-2, bf16, early-stop rule
    live (patience past the run), graph-replayed chunks of 16 rounds."""
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    cfg = EngineConfig(hidden=(50, 200), max_rounds=rounds + 40, early_stop=True, patience=rounds + 41,
                       dtype="bf16", graph_rounds=16, lagged_eval=lagged)
    e = HipRoundEngine(X, y, 2, cfg, comm, flat, n_total=n_total)
    info = {"adam_exchange": bool(e.engine.adam_exchange), "lagged": bool(e.engine.lagged),
            "adam_grid": int(e._peer.adam_grid) if e._peer is not None else -1,
            "uses_ll": bool(e._peer.uses_ll) if e._peer is not None else False,
            "uses_rsag": bool(e._peer.uses_rsag) if e._peer is not None else False, "R": e.R}
    e.run(rounds)
    e.sync_history()
    out = (e.global_flat(), e.history(), e.local_flat(), info)
    del e
    return out


def _worker_prod(rank, world, port, rounds, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import gc
        import torch
        from bench import reference_rows, synth_shard
        from fedmi.models.mlp import init_flat
        from fedmi.parallel.comm import Comm
        # RCCL allowed: the xgmi plane must never bootstrap it while the peer plane works
        comm = Comm(backend="xgmi", device="cuda:0", rccl=True)
        dev = comm.device
        rows = reference_rows(8000, world, rank)           # 1000 rows per client at world 8
        X, y = synth_shard(rows, rank, dev)
        flat = init_flat([14, 50, 200, 2], seed=rank)
        res = {}
        res["ll"] = _run_prod(comm, X, y, flat, 8000, True, rounds)
        gc.collect()
        os.environ["FEDMI_PEER_LL"] = "0"                   # publish / wait / pull weight chunks
        try:
            res["pull"] = _run_prod(comm, X, y, flat, 8000, True, rounds)
        finally:
            del os.environ["FEDMI_PEER_LL"]
        gc.collect()
        os.environ["FEDMI_PEER_RSAG"] = "1"                 # reduce-scatter + all-gather weight chunks
        try:
            res["rsag"] = _run_prod(comm, X, y, flat, 8000, True, rounds)
        finally:
            del os.environ["FEDMI_PEER_RSAG"]
        gc.collect()
        res["classic"] = _run_prod(comm, X, y, flat, 8000, False, rounds)   # standalone peer kernel
        res["rccl_created"] = comm.native is not None
        torch.cuda.synchronize()
        comm.Barrier()
        q.put((rank, res, None))
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(900)
def test_peer_world8_production_shape_adam_exchange():
    """SCALE's default N = 8 round before any 8-GPU node runs it: 8 ranks (sharing cuda:0),
    the reference model 14-50-200-2 on the reference's 1000-row shards, lagged evaluation with
    FedAvg inside the Adam kernel (LL chunks, and publish / wait / pull chunks), early-stop
    rule live, 64 graph-replayed rounds: bit-identical weights, history and per-client metrics
    to classic rounds over the standalone peer kernel.  The shared GPU cannot hold 8 full Adam
    grids (8 x 179 spinning 1024-thread blocks), so the exchange runs on the bounded grid
    (peer.shared_adam_grid -> 16 workgroups per rank, fl_adam_ll_grid_kernel) -- the same
    per-block computation.  RCCL is allowed but never bootstrapped (the xgmi plane is lazy)."""
    world, rounds = 8, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_prod, args=(r, world, port, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=800) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, res, err in out:
        assert err is None, f"rank {rank}:\n{err}"
        (wl, hl, ll, il), (wp, hp, lp, ip), (wc, hc, lc, ic) = res["ll"], res["pull"], res["classic"]
        (wr, hr, lr, ir) = res["rsag"]
        assert il["adam_exchange"] and il["uses_ll"] and not il["uses_rsag"] and il["adam_grid"] == 16, il
        assert ip["adam_exchange"] and not ip["uses_ll"] and ip["adam_grid"] == 16, ip  # fl_adam_grid_kernel
        assert ir["adam_exchange"] and ir["uses_rsag"] and ir["adam_grid"] == 16, ir    # fl_adam_rsag_grid_kernel
        assert not ic["adam_exchange"] and not ic["lagged"], ic
        assert not res["rccl_created"]
        assert hl["rounds_run"] == hc["rounds_run"] == rounds and hl["stop_round"] < 0
        for name, (w, h, lo) in (("ll", (wl, hl, ll)), ("pull", (wp, hp, lp)), ("rsag", (wr, hr, lr))):
            np.testing.assert_array_equal(w, wc, err_msg=f"rank {rank} {name}: global weights")
            np.testing.assert_array_equal(lo, lc, err_msg=f"rank {rank} {name}: local weights")
            np.testing.assert_array_equal(h["global"], hc["global"], err_msg=f"rank {rank} {name}: metrics")
            np.testing.assert_array_equal(h["per_rank"], hc["per_rank"])
            np.testing.assert_array_equal(h["loss"], hc["loss"])
    for r in range(1, world):
        np.testing.assert_array_equal(out[0][1]["ll"][0], out[r][1]["ll"][0])
