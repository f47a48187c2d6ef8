"""Bounded, agreed RCCL bootstrap (``Comm.rccl`` in fedmi/parallel/comm.py).

The reference's failure contract is "any exception -> comm.Abort()"
(FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:203-205): a rank must never be left
blocked because a peer died.  ``Comm.rccl()`` shares the RCCL unique id through the gloo store
with a deadline, runs the (non-blocking, deadline-bounded) native init, and then has every rank
post its outcome and wait -- bounded -- for everyone else's.  These CPU tests (gloo, world 2)
replace the native init with a fake so every failure shape runs here:

* both ranks succeed -> both hold a communicator;
* one rank's init fails -> BOTH ranks raise, naming that rank, and the surviving handle is aborted;
* one rank never calls the bootstrap at all -> the other raises within the deadline instead of
  hanging (root and non-root variants);
* gloo / ``rccl=False`` never create one (the xgmi plane's laziness is a GPU test:
  tests/test_peer_allreduce.py::test_xgmi_plane_never_bootstraps_rccl).

The native side (ncclCommInitRankConfig, blocking = 0, ncclCommAbort on timeout) is covered on
the GPU by tests/test_rccl.py::test_rccl_bootstrap_times_out_when_peer_never_joins.
"""
import os
import socket
import time

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeHandle:
    def __init__(self, uid):
        self.uid, self.aborted = uid, False

    def abort(self):
        self.aborted = True


def _make_factory(mode, rank):
    def factory(uid):
        if mode == "fail" and rank == 1:
            raise RuntimeError("simulated ncclCommInitRankConfig failure")
        return _FakeHandle(uid)
    factory.unique_id = lambda: b"U" * 128
    return factory


def _worker(rank, world, port, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.set_num_threads(1)
    from fedmi.parallel.comm import Comm
    comm = Comm(backend="gloo", device="cpu", rccl_timeout_s=3.0)
    comm.rccl_allowed = True
    comm._rccl_factory = _make_factory(mode, rank)
    out = {"rank": rank}
    if mode == "shared":
        # two ranks on one GPU (device identities equal): the native bootstrap is never reached
        import fedmi.parallel.peer as peer
        peer.device_key = lambda device: "gpu-0-uuid"
        comm.device = torch.device("cuda", 0)
        comm._rccl_factory = None
        out["handle"] = comm.rccl()
        out["allowed"] = comm.rccl_allowed
        # rank 0 hosts the store: it leaves only after the other rank has finished with it
        store = comm._store()
        if rank != 0:
            store.set("test/done/1", "1")
        else:
            t_end = time.monotonic() + 30.0
            while not store.check(["test/done/1"]) and time.monotonic() < t_end:
                time.sleep(0.01)
        q.put(out)
        q.close()
        q.join_thread()
        os._exit(0)
    if mode == "fallback":
        # FEDMI_TEST_RCCL_FAIL=1: rank 1's bootstrap fails -> EVERY rank lands on the host plane,
        # RCCL is disabled for the rest of the job, and the next device all-reduce works (host)
        os.environ["FEDMI_TEST_RCCL_FAIL"] = "1"
        out["handle"] = comm.rccl_or_host()
        out["allowed"] = comm.rccl_allowed
        out["error"] = comm.rccl_error
        out["again"] = comm.rccl()          # no second bootstrap
        t = torch.full((5,), float(rank + 1))
        comm.allreduce_(t)
        out["sum"] = t.tolist()
        # the host plane of device buffers sums in rank order (left fold, bit-identical to the
        # xGMI kernels): fp32 values whose sum depends on the order
        v = torch.tensor([1e8, 1.0, -1e8, 3.0], dtype=torch.float32)[rank:rank + 1].repeat(3)
        out["ordered"] = comm._host_sum_rank_order(v).tolist()
        q.put(out)
        q.close()
        q.join_thread()
        os._exit(0)
    absent = {"absent1": 1, "absent0": 0}.get(mode)
    t0 = time.monotonic()
    if rank == absent:
        # this rank never joins the bootstrap; it outlives the peer's deadline, then leaves
        time.sleep(12.0)
        out["skipped"] = True
    else:
        try:
            h = comm.rccl()
            out["ok"] = h is not None and h.uid == b"U" * 128
            out["cached"] = comm.rccl() is h   # second call: no new bootstrap
        except Exception as e:  # noqa: BLE001
            out["err"] = f"{type(e).__name__}: {e}"
            out["handle_aborted"] = getattr(comm, "native", None) is None
    out["elapsed"] = time.monotonic() - t0
    q.put(out)
    q.close()
    q.join_thread()  # flush the queue's feeder thread before the hard exit
    # leave without the gloo teardown handshake (the absent rank's peer may be gone)
    os._exit(0)


def _run(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda d: d["rank"])
    for p in procs:
        p.join(timeout=60)
    return res


def test_bootstrap_agreed_success():
    res = _run("ok")
    assert all(r.get("ok") and r.get("cached") for r in res), res


def test_bootstrap_one_rank_fails_both_raise():
    res = _run("fail")
    for r in res:
        assert "RCCL bootstrap failed on rank 1" in r.get("err", ""), res
        assert "simulated" in r["err"]
        assert r["handle_aborted"]


@pytest.mark.parametrize("mode", ["absent1", "absent0"])
def test_bootstrap_peer_never_arrives_raises_within_deadline(mode):
    res = _run(mode)
    live = [r for r in res if not r.get("skipped")]
    assert len(live) == 1
    r = live[0]
    # rank 0 (root) waits for the outcome of the never-arriving rank 1; rank 1 waits for the
    # unique id that never-arriving rank 0 would publish -- both name what they waited for
    assert "err" in r, res
    assert ("rank(s) [1]" in r["err"]) if mode == "absent1" else ("rank 0 did not publish" in r["err"])
    assert r["elapsed"] < 10.0, r   # deadline 3 s (+3 s agreement), not gloo's 600 s


def test_bootstrap_skipped_when_ranks_share_a_gpu():
    """Ranks whose devices are the same GPU (``--device cuda:0`` on a one-GPU box) agree over the
    store to stay on the host path: RCCL refuses duplicate devices, so no bootstrap is attempted."""
    res = _run("shared")
    for r in res:
        assert r["handle"] is None and r["allowed"] is False, res


def test_rccl_not_allowed_returns_none():
    """gloo (and ``rccl=False``) never bootstrap RCCL: ``rccl()`` is None, device all-reduces
    then go through the host."""
    from fedmi.parallel.comm import Comm
    c = Comm(backend="gloo", device="cpu")
    assert c.native is None and c.rccl() is None and not c.rccl_allowed


def test_failed_bootstrap_falls_back_to_host_on_every_rank():
    """Data-plane fallback chain, last link: when the RCCL bootstrap fails on one rank, every
    rank gets ``None`` from ``rccl_or_host`` (the outcome is agreed), RCCL stays disabled, and
    device all-reduces continue on the host plane with rank-order sums (world 4)."""
    res = _run("fallback", world=4)
    for r in res:
        assert r["handle"] is None and r["allowed"] is False and r["again"] is None, res
        assert "rank 1" in r["error"] and "FEDMI_TEST_RCCL_FAIL" in r["error"], r
        assert r["sum"] == [10.0] * 5
        # ((1e8 + 1) + -1e8) + 3 in fp32 = 3 (the 1 is lost), not 4 = any order adding 1 last
        assert r["ordered"] == [3.0] * 3, r
