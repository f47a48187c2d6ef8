"""The engine-owned RCCL communicator (``RcclComm`` in fedmi/ops/csrc/fl_engine.cpp) on the
one-GPU box: RCCL cannot put two ranks on one device, so these run a ONE-rank communicator --
every call still goes through ``ncclCommInitRank`` / ``ncclAllReduce`` / ``ncclBroadcast`` /
``ncclAllGather`` on a real stream, eagerly and inside captured HIP graphs:

* raw collectives (f32 / f64 / bf16 all-reduce, byte broadcast, all-gather), eager and
  captured;
* the fused round engine issuing its FedAvg all-reduce through RCCL (an emulating engine:
  ``emulate_clients`` keeps the multi-client round shape at world 1), eager and inside
  ``FLEngine.capture``: bit-identical to the same engine without a collective (a one-rank
  SUM is the identity);
* the wide client's per-layer FedAvg buckets through ``Comm.allreduce_`` -> RCCL.

The multi-rank RCCL path itself is exercised by the driver's 8-GPU scaling run
(``bench.py --backend rccl`` / ``FEDMI_DATA_PLANE=rccl``).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rccl():
    import torch
    from fedmi.ops import native
    m = native()
    torch.cuda.set_device(0)
    return m, m.RcclComm(1, 0, m.RcclComm.unique_id(), 0)


def test_rccl_raw_collectives_eager_and_graph():
    import torch
    m, rc = _rccl()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    x = torch.randn(50003, device=dev)
    ref = x.clone()
    xd = torch.randn(1001, dtype=torch.float64, device=dev)
    refd = xd.clone()
    b = torch.arange(256, dtype=torch.uint8, device=dev)
    out = torch.empty_like(x)
    with torch.cuda.stream(s):
        rc.allreduce_f32(x.data_ptr(), x.numel(), s.cuda_stream)
        rc.allreduce_f64(xd.data_ptr(), xd.numel(), s.cuda_stream)
        rc.broadcast_bytes(b.data_ptr(), b.numel(), 0, s.cuda_stream)
        rc.allgather_f32(x.data_ptr(), out.data_ptr(), x.numel(), s.cuda_stream)
    s.synchronize()
    assert torch.equal(x, ref) and torch.equal(xd, refd) and torch.equal(out, ref)
    assert torch.equal(b.cpu(), torch.arange(256, dtype=torch.uint8))
    xb = torch.randn(40001, device=dev).to(torch.bfloat16)
    refb = xb.clone()
    with torch.cuda.stream(s):
        rc.allreduce_bf16(xb.data_ptr(), xb.numel(), s.cuda_stream)
    s.synchronize()
    assert torch.equal(xb, refb)
    # captured: all-reduce of a buffer that a captured kernel rewrites before every replay
    g = torch.cuda.CUDAGraph()
    y = torch.zeros(4096, device=dev)
    with torch.cuda.graph(g, stream=s):
        y.add_(1.0)
        rc.allreduce_f32(y.data_ptr(), y.numel(), torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert float(y.min()) == float(y.max()) == 3.0  # capture does not execute: 3 replays
    rc.destroy()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_round_engine_fedavg_through_rccl(dtype):
    """The engine's RCCL path (issue_allreduce -> ncclAllReduce), eager + graph-captured rounds."""
    import torch
    from fedmi.data.synthetic import make_income_like
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    m, rc = _rccl()
    X, y = make_income_like(2000, seed=3)
    flat = init_flat([14, 50, 200, 2], 1)
    res = []
    for use_rccl in (True, False):
        cfg = EngineConfig(max_rounds=40, early_stop=False, dtype=dtype, graph_rounds=4, fused_eval=False)
        e = HipRoundEngine(X, y, 2, cfg, None, flat, emulate_clients=True)
        if use_rccl:
            e._native_comm = rc
        e.run(3)          # eager
        e.run(13)         # graph chunks (capture passes the communicator)
        e.sync_history()
        assert e.history()["rounds_run"] == 16
        res.append((e.global_flat(), e.history()["global"], e.history()["loss"]))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][2], res[1][2])
    torch.cuda.synchronize()
    rc.destroy()


@pytest.mark.parametrize("check_every,seed", [(2, 6), (2, 7), (7, 6), (64, 6), (64, 8)])
def test_lagged_rounds_with_early_stop_over_rccl(check_every, seed):
    """Lagged rounds with early stopping when the FedAvg rides RCCL: region
    A is folded one round late, so the round after the stop's trigger has already run when the
    stop is found -- by the next Adam kernel or by the finalize kernel (``check_every`` 2: every
    other round closes a host chunk) -- and is discarded.  Weights, metric history, loss and the
    stop round are bitwise equal to classic rounds (a separate evaluation per round) over the same
    one-rank RCCL communicator -- and so are the local model, the Adam moments and the local
    evaluation, which the discarded round's step had already changed."""
    import torch
    from fedmi.data.synthetic import make_income_like
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    m, rc = _rccl()
    X, y = make_income_like(3000, seed=11)
    flat = init_flat([14, 50, 200, 2], seed)
    res = []
    for lag in (True, False):
        cfg = EngineConfig(max_rounds=300, patience=4, tolerance=2e-3, dtype="bf16", fused_eval=False,
                           lagged_eval=lag, graph_rounds=4)
        e = HipRoundEngine(X, y, 2, cfg, None, flat, emulate_clients=True)
        e._native_comm = rc
        assert e.engine.lagged == lag and e.engine.late_fold == lag
        e.run(300, check_every=check_every)
        h = e.history()
        st = e.portable_state()
        res.append((e.global_flat(), h, e.engine.eval_launches, e.local_flat(), st, e.confusion()))
    (wl, hl, ev_l, ll, sl, cl), (wc, hc, ev_c, lc, sc, cc) = res
    assert hc["stop_round"] > 0, "the classic run must stop early for this test to mean anything"
    assert hl["stop_round"] == hc["stop_round"] and hl["rounds_run"] == hc["rounds_run"]
    np.testing.assert_array_equal(wl, wc)
    np.testing.assert_array_equal(hl["global"], hc["global"])
    np.testing.assert_array_equal(hl["per_rank"], hc["per_rank"])
    np.testing.assert_array_equal(hl["loss"], hc["loss"])
    # the discarded round's local step is undone too (FLBuffers::undo): local model,
    # Adam moments and the local evaluation match the run that stopped in time
    np.testing.assert_array_equal(ll, lc)
    for k in ("exp_avg", "exp_avg_sq"):
        np.testing.assert_array_equal(np.asarray(sl[k]), np.asarray(sc[k]), err_msg=k)
    np.testing.assert_array_equal(cl, cc)
    # lagged rounds evaluate only the closing round of each host chunk
    assert ev_l < ev_c
    torch.cuda.synchronize()
    rc.destroy()


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_wide_aggregate_through_rccl(wire):
    """WideClient.aggregate: per-layer buckets all-reduced as n_i/N-scaled sums on the comm
    stream, fp32 or bf16 on the wire (one rank: the scale is 1, so the weights must come back
    unchanged -- bf16: up to one bf16 rounding of the round's update)."""
    import torch
    from fedmi.data.synthetic import make_income_like
    from fedmi.fl.wide import WideClient
    m, rc = _rccl()
    dev = torch.device("cuda", 0)
    Xn, yn = make_income_like(1024, seed=5)
    X, y = torch.as_tensor(Xn, device=dev), torch.as_tensor(yn, device=dev)
    c = WideClient(X, y, [14, 256, 128, 2], comm=None, micro_batch=512, dtype="bf16")
    g0 = c.params.clone()   # the global model this local step started from
    c.local_step()
    c.stream.synchronize()
    before = c.params.clone()
    # force the multi-client aggregate path with the one-rank RCCL communicator
    c.world, c.comm = 2, _OneRankDevComm(rc)
    if wire == "bf16":
        c.send_bf16 = torch.empty(c.params.numel(), dtype=torch.bfloat16, device=dev)
        c.gprev = g0.clone()
    c.aggregate()
    c.sync()
    torch.cuda.synchronize()
    assert c.comm.calls == c.L and c.comm.scales == ([c.agg] if wire == "fp32" else [None]) * c.L
    if wire == "fp32":
        assert torch.equal(c.params, before)
    else:
        # the round's delta crosses the wire as bf16 and is added back to the fp32 global model
        expect = g0 + (before - g0).to(torch.bfloat16).float()
        assert torch.equal(c.params, expect)
        assert torch.equal(c.gprev, expect)
    rc.destroy()


class _OneRankDevComm:
    """Comm stand-in whose device all-reduce is the one-rank RCCL communicator."""

    def __init__(self, rc):
        self.rc, self.calls, self.size, self.rank, self.scales = rc, 0, 1, 0, []

    def allreduce_(self, t, scale=None):
        import torch
        s = torch.cuda.current_stream(t.device).cuda_stream
        if scale is not None:
            t.mul_(scale)
        if t.dtype == torch.bfloat16:
            self.rc.allreduce_bf16(t.data_ptr(), t.numel(), s)
        else:
            self.rc.allreduce_f32(t.data_ptr(), t.numel(), s)
        self.calls += 1
        self.scales.append(scale)
        return t


_BOOT_CHILD = r"""
import sys, time
import torch
from fedmi.ops import native
m = native()
torch.cuda.set_device(0)
rank = int(sys.argv[1])
uid = m.RcclComm.unique_id()
t0 = time.monotonic()
try:
    m.RcclComm(2, rank, uid, 0, 5.0)
    print("NO_RAISE", flush=True)
except RuntimeError as e:
    print(f"RAISED {time.monotonic() - t0:.2f} {e}", flush=True)
# the process is still usable: a fresh one-rank communicator all-reduces
rc = m.RcclComm(1, 0, m.RcclComm.unique_id(), 0)
x = torch.arange(1000, dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
rc.allreduce_f32(x.data_ptr(), x.numel(), s)
torch.cuda.synchronize()
print("AFTER_OK" if torch.equal(x.cpu(), torch.arange(1000, dtype=torch.float32)) else "AFTER_BAD", flush=True)
rc.destroy()
"""


@pytest.mark.timeout(240)
@pytest.mark.parametrize("rank", [0, 1])
def test_rccl_bootstrap_times_out_when_peer_never_joins(rank):
    """A world-2 RCCL bootstrap whose other rank never calls init (rank 0 = the unique-id root,
    rank 1 = a joining rank whose root never arrives): the non-blocking ncclCommInitRankConfig is
    polled against the 5 s deadline with the GIL released, aborted, and raises a clear error --
    instead of blocking in ncclCommInitRank forever (reference contract: any failure ->
    comm.Abort(), C:203-205).  Run in a child process under its own time limit, so a
    regression shows up as a failed test, not a hung session."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _BOOT_CHILD, str(rank)], cwd=root, capture_output=True, text=True,
                       timeout=180)
    out = p.stdout
    assert p.returncode == 0, (p.returncode, out, p.stderr[-3000:])
    line = next((x for x in out.splitlines() if x.startswith(("RAISED", "NO_RAISE"))), "")
    assert line.startswith("RAISED"), (out, p.stderr[-3000:])
    elapsed = float(line.split()[1])
    assert "timed out" in line and elapsed < 30.0, line
    assert "AFTER_OK" in out, out
