"""Fail-fast xGMI data plane and the data-plane fallback chain.

The reference's failure contract is "any exception -> comm.Abort()"
(FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:129,203-205); its MPI gathers would
block forever on a dead rank.  On the default GPU data plane every device wait is bounded
(``$FEDMI_PEER_TIMEOUT_S``), a timeout writes a sticky failure word into EVERY rank's control
block (so each later wait of every rank returns at once and the whole job drains in one
timeout), a host abort word lets ``Comm.Abort`` / watchdogs release spinning kernels and tell the
peers, and the round engine checks the word after every chunk of rounds -- before the chunk is
printed -- then aborts.

GPU cases share ``cuda:0`` between the ranks (the one-GPU box): the peer protocol runs unchanged
between processes of one device.
"""
import os
import re
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(REPO, "FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---------------------------------------------------------------------------------------------
# CPU: decoding of the failure word, timeout knob
# ---------------------------------------------------------------------------------------------
def test_describe_peer_error():
    from fedmi.parallel.peer import describe_peer_error
    assert describe_peer_error((1 << 16) | (0 << 8) | 1, 5.0) == "rank 0 waited 5 s for rank 1, which died or stalled"
    assert describe_peer_error((2 << 16) | (3 << 8) | 0xFF) == "rank 3 aborted the job"
    assert "evaluation blocks" in describe_peer_error((1 << 16) | (2 << 8) | 0xFE, 1.0)


def test_peer_timeout_knob(monkeypatch):
    from fedmi.parallel.peer import DEFAULT_PEER_TIMEOUT_S, peer_timeout_s
    monkeypatch.delenv("FEDMI_PEER_TIMEOUT_S", raising=False)
    assert peer_timeout_s() == DEFAULT_PEER_TIMEOUT_S
    monkeypatch.setenv("FEDMI_PEER_TIMEOUT_S", "7.5")
    assert peer_timeout_s() == 7.5
    assert peer_timeout_s(3.0) == 3.0


def test_check_peer_error_raises():
    from fedmi.parallel.peer import PeerFailure, check_peer_error

    class _H:
        timeout_s = 4.0

        def __init__(self, w):
            self.w = w

        def error(self):
            return self.w
    check_peer_error(None)
    check_peer_error(_H(0))
    with pytest.raises(PeerFailure, match="rank 1 waited 4 s for rank 0"):
        check_peer_error(_H((1 << 16) | (1 << 8) | 0))


def test_fault_keeps_every_rank_on_the_same_chunking(monkeypatch):
    """Every rank ends a run call at the fault round (the chunking -- and so each round's
    collectives -- stays identical); only the faulting rank fails there."""
    from fedmi.fl.trainer import FederatedMLPLearning
    from fedmi.runtime.fault import FaultSpec

    calls = {}

    class _Eng:
        def __init__(self):
            self.rounds_issued, self.stopped = 0, False
            self.cfg = type("C", (), {"patience": 10, "tolerance": 1e-4})()
            self.hist = type("H", (), {"rounds_run": 0, "global_metrics_dict": lambda s: {}})()
            self.dims = [14, 4, 2]

        def run_streaming(self, n, chunk, on_history, guard):
            calls.setdefault("n", []).append(n)
            self.rounds_issued += n
            return n

    for rank in (0, 1):
        calls.clear()
        tr = FederatedMLPLearning.__new__(FederatedMLPLearning)
        tr.rank, tr.engine, tr.comm = rank, _Eng(), None
        fault = FaultSpec(1, 40, "raise")
        if rank == 1:
            with pytest.raises(Exception, match="injected fault"):
                tr.train_and_evaluate(None, rounds=300, fault=fault, verbose=True)
            assert calls["n"] == [40]
        else:
            tr.engine.global_flat = lambda: np.zeros(3)
            import fedmi.fl.trainer as T
            monkeypatch.setattr(T, "flat_to_dict", lambda flat, dims: {})
            tr.train_and_evaluate(None, rounds=300, fault=fault, verbose=True)
            assert calls["n"] == [40, 260]


# ---------------------------------------------------------------------------------------------
# GPU: raw communicator -- a rank that never joins; propagation; host abort
# ---------------------------------------------------------------------------------------------
def _worker_raw(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch
        from fedmi.parallel.comm import Comm
        from fedmi.parallel.peer import describe_peer_error, make_peer_allreduce
        comm = Comm(backend="xgmi", device="cuda:0", rccl=False)
        dev = comm.device
        s = torch.cuda.current_stream(dev)
        out = torch.empty(4096, device=dev)
        res = {}
        # 1. rank 1 never calls: rank 0's kernel ends after ~2 s and reports rank 1 on BOTH ranks
        h = make_peer_allreduce(comm, 4096, dev, timeout_s=2.0)
        assert h is not None
        if rank == 0:
            t0 = time.monotonic()
            h.allreduce(0, out.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
            res["wait_s"] = time.monotonic() - t0
        comm.Barrier()
        w = int(h.error())
        res["word"], res["desc"] = w, describe_peer_error(w, 2.0)
        # 2. later calls of a failed communicator return at once (the sticky word ends every wait)
        if rank == 0:
            t0 = time.monotonic()
            for k in range(5):
                h.allreduce(k & 1, out.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
            res["after_s"] = time.monotonic() - t0
        comm.Barrier()
        h.close()
        # 3. host abort: rank 0 spins (60 s timeout) until its host aborts from another thread
        h = make_peer_allreduce(comm, 4096, dev, timeout_s=60.0)
        if rank == 0:
            t0 = time.monotonic()
            h.allreduce(0, out.data_ptr(), s.cuda_stream)
            threading.Timer(1.0, lambda: res.__setitem__("told", bool(h.abort(2.0)))).start()
            torch.cuda.synchronize(dev)
            res["abort_wait_s"] = time.monotonic() - t0
            time.sleep(0.5)
        comm.Barrier()
        res["abort_word"] = int(h.error())
        comm.Barrier()
        h.close()
        q.put((rank, res, None))
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_device_wait_times_out_propagates_and_host_abort_releases():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_raw, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, res, err in out:
        assert err is None, f"rank {rank}:\n{err}"
        # the timeout is reported by rank 0, naming rank 1, in BOTH ranks' words
        assert res["word"] == (1 << 16) | (0 << 8) | 1, (rank, hex(res["word"]))
        assert res["desc"] == "rank 0 waited 2 s for rank 1, which died or stalled"
        assert res["abort_word"] == (2 << 16) | (0 << 8) | 0xFF, (rank, hex(res["abort_word"]))
    r0 = out[0][1]
    assert 1.9 < r0["wait_s"] < 8.0, r0
    assert r0["after_s"] < 1.0, r0          # five more calls: no second timeout
    assert r0["told"] is True and 0.9 < r0["abort_wait_s"] < 10.0, r0


# ---------------------------------------------------------------------------------------------
# GPU: a client dies / hangs / raises at round 40 of a 300-round [C] run (HIP engine, xGMI plane)
# ---------------------------------------------------------------------------------------------
class _Proc:
    def __init__(self, rank, port, args, env):
        e = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(port), PYTHONPATH=REPO, PYTHONUNBUFFERED="1", **env)
        self.p = subprocess.Popen([sys.executable, ENTRY, *args], cwd=REPO, env=e, stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True)
        self.lines = []   # (time, line)
        self.t = threading.Thread(target=self._read, daemon=True)
        self.t.start()

    def _read(self):
        for line in self.p.stdout:
            self.lines.append((time.monotonic(), line.rstrip("\n")))

    def first(self, pat):
        for t, l in self.lines:
            if re.search(pat, l):
                return t
        return None

    def text(self):
        return "\n".join(l for _, l in self.lines)


@pytest.mark.gpu
@pytest.mark.timeout(420)
@pytest.mark.parametrize("kind,dtype", [("exit", "bf16"), ("hang", "bf16"), ("raise", "bf16"), ("exit", "fp32")])
def test_dead_client_aborts_the_job_within_the_peer_timeout(kind, dtype):
    """bf16: lagged rounds, FedAvg inside the Adam kernel (LL exchange); fp32: evaluation +
    FedAvg kernel (publish / wait / pull).  The host watchdog is off: the device path alone
    must end the job."""
    timeout_s = 5.0
    port = _free_port()
    args = ["--device", "cuda:0", "--rounds", "300", "--no-early-stop", "--fault-inject", f"1:40:{kind}",
            "--peer-timeout-s", str(timeout_s), "--watchdog-s", "0", "--dtype", dtype]
    procs = [_Proc(r, port, args, {}) for r in range(2)]
    try:
        rc0 = procs[0].p.wait(timeout=360)
        t_end = time.monotonic()
    finally:
        for p in procs:
            if p.p.poll() is None:
                p.p.kill()
            p.p.wait(timeout=30)
            p.t.join(timeout=10)
    out0, out1 = procs[0].text(), procs[1].text()
    t_fault = procs[1].first(r"injected fault")
    assert t_fault is not None, out1[-3000:]
    assert rc0 != 0, out0[-3000:]
    assert "Rank 0 encountered an error: xGMI data plane failed" in out0, out0[-3000:]
    if kind == "raise":
        assert "rank 1 aborted the job" in out0, out0[-3000:]     # told by rank 1's Comm.Abort
    else:
        assert "rank 0 waited 5 s for rank 1" in out0, out0[-3000:]
    assert t_end - t_fault < timeout_s + 15.0, (t_end - t_fault)
    # rounds 1..40 were printed (both clients contributed); nothing after them passes as valid
    rounds = [int(m) for m in re.findall(r"Global Metrics \(Round (\d+)\)", out0)]
    assert rounds and max(rounds) == 40, rounds[-5:]
    err = [l for l in out0.splitlines() if "encountered an error" in l][0]
    print(f"\n[fail-fast] {kind}/{dtype}: rank 0 exit status {rc0}, {t_end - t_fault:.2f} s after rank 1's fault "
          f"(peer timeout {timeout_s:g} s); last round printed {max(rounds)}; {err.strip()}")


# ---------------------------------------------------------------------------------------------
# GPU: the fallback chain -- peer set-up fails on rank 1 -> every rank on the next plane
# ---------------------------------------------------------------------------------------------
def _run_rounds(comm, X, y, flat, rounds):
    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    cfg = EngineConfig(hidden=(50, 200), max_rounds=rounds + 40, early_stop=True, patience=rounds + 41,
                       dtype="bf16", graph_rounds=16)
    e = HipRoundEngine(X, y, 2, cfg, comm, flat, n_total=8000)
    agg = e.aggregation
    e.run(rounds)
    e.sync_history()
    out = (agg, e.global_flat(), e.history(), e.local_flat())
    del e
    return out


def _worker_fallback(rank, world, port, rounds, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import gc
        import torch
        from bench import reference_rows, synth_shard
        from fedmi.models.mlp import init_flat
        from fedmi.parallel.comm import Comm
        comm = Comm(backend="xgmi", device="cuda:0", rccl=True)
        dev = comm.device
        X, y = synth_shard(reference_rows(8000, world, rank), rank, dev)
        flat = init_flat([14, 50, 200, 2], seed=rank)
        res = {"peer": _run_rounds(comm, X, y, flat, rounds)}
        gc.collect()
        os.environ["FEDMI_TEST_PEER_FAIL"] = "1"      # rank 1's peer set-up fails
        try:
            res["fallback"] = _run_rounds(comm, X, y, flat, rounds)
        finally:
            del os.environ["FEDMI_TEST_PEER_FAIL"]
        torch.cuda.synchronize()
        comm.Barrier()
        q.put((rank, res, None))
        comm.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_peer_setup_failure_lands_every_rank_on_the_host_plane(world):
    """FEDMI_TEST_PEER_FAIL=1: rank 1's peer set-up fails.  Every rank agrees to fall back; RCCL
    cannot put ranks of one GPU on a communicator, so every rank lands on the HOST plane (gloo,
    rank-order sums) and the run is bit-identical to the peer plane's."""
    import torch.multiprocessing as mp
    rounds = 48
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_fallback, args=(r, world, port, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=500) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    for rank, res, err in out:
        assert err is None, f"rank {rank}:\n{err}"
        (ap, wp, hp, lp), (af, wf, hf, lf) = res["peer"], res["fallback"]
        assert ap == "xgmi-oneshot+adam" and af == "host", (ap, af)
        assert hp["rounds_run"] == hf["rounds_run"] == rounds
        np.testing.assert_array_equal(wf, wp, err_msg=f"rank {rank}: global weights")
        np.testing.assert_array_equal(lf, lp, err_msg=f"rank {rank}: local weights")
        np.testing.assert_array_equal(hf["global"], hp["global"])
        np.testing.assert_array_equal(hf["per_rank"], hp["per_rank"])
        np.testing.assert_array_equal(hf["loss"], hp["loss"])


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_labels_the_host_plane():
    """bench.py --gpus 2 --share-gpu with rank 1's peer set-up failing still prints ONE record,
    labelled data_plane 'host' with a warning."""
    import json
    env = dict(os.environ, FEDMI_TEST_PEER_FAIL="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--share-gpu", "--steps", "20", "--warmup", "5",
                        "--no-convergence", "--no-anchor", "--no-weak"], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["config"]["data_plane"] == "host" and "HOST plane" in rec["warning"], rec
    assert rec["replicas_consistent"] is True and rec["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_reruns_on_the_next_plane_after_a_peer_failure():
    """A failure reported on the xGMI plane during the headline's rounds (FEDMI_TEST_PEER_ERROR=1:
    one simulated report on every rank) does not end the bench without a number: every rank re-runs
    the timed rounds on the next plane (ranks sharing a GPU: the host) and the record says so."""
    import json
    env = dict(os.environ, FEDMI_TEST_PEER_ERROR="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--share-gpu", "--steps", "20", "--warmup", "5",
                        "--no-convergence", "--no-anchor", "--no-weak"], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert "xGMI data plane failed" in rec["data_plane_failure"], rec
    assert rec["config"]["data_plane"] == "host" and rec["replicas_consistent"] is True and rec["value"] > 0
