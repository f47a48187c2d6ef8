"""Abort path, collective watchdog and entrypoint-level resume.

Multi-process cases run the real [C] entrypoint under ``torch.distributed.run`` with 2 CPU
clients on gloo (BASELINE config 1), with one client failing at round 3."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from fedmi.runtime.fault import FaultSpec, InjectedFault, parse_fault
from fedmi.runtime.watchdog import Watchdog

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(REPO, "FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py")
DATA = os.path.join(REPO, "data", "balanced_income_data.csv")


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(args, nproc=2, timeout=150):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), ENTRY, "--device", "cpu",
           "--backend", "gloo", "--engine", "torch", "--data", DATA, *args]
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    t0 = time.time()
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr, time.time() - t0


def test_parse_fault():
    assert parse_fault("1:3") == FaultSpec(1, 3, "raise")
    assert parse_fault("0:7:hang").kind == "hang"
    assert parse_fault(None) is None
    with pytest.raises(ValueError):
        parse_fault("1:3:explode")
    with pytest.raises(InjectedFault):
        FaultSpec(0, 1).trigger(0, 1)


def test_watchdog_fires_and_disarms():
    fired = []
    wd = Watchdog(0.3, lambda: fired.append(1))
    with wd.guard("fast"):
        time.sleep(0.05)
    time.sleep(0.5)
    assert not fired
    with wd.guard("slow"):
        time.sleep(0.8)
    assert fired and wd.fired
    wd.close()


@pytest.mark.parametrize("kind", ["raise", "exit"])
def test_client_failure_tears_down_the_job(kind):
    rc, out, dt = _torchrun(["--rounds", "8", "--fault-inject", f"1:3:{kind}", "--no-early-stop"])
    assert rc != 0
    assert "injected fault" in out
    if kind == "raise":
        assert "Rank 1 encountered an error" in out   # reference C:203-205 message
    assert dt < 120


def test_hung_client_is_caught_by_watchdog():
    rc, out, dt = _torchrun(["--rounds", "8", "--fault-inject", "1:3:hang", "--no-early-stop",
                             "--watchdog-s", "4"])
    assert rc != 0
    assert "[watchdog] rank 0" in out
    assert dt < 120


def test_entrypoint_resume_matches_straight_run(tmp_path):
    base = ["--rounds", "12", "--no-early-stop", "--quiet"]
    rc, out, _ = _torchrun([*base, "--jsonl", str(tmp_path / "a.jsonl")])
    assert rc == 0, out
    ck = str(tmp_path / "ck")
    rc, out, _ = _torchrun(["--rounds", "5", "--no-early-stop", "--quiet", "--save", ck])
    assert rc == 0, out
    rc, out, _ = _torchrun([*base, "--resume", ck, "--jsonl", str(tmp_path / "b.jsonl")])
    assert rc == 0, out
    assert "Resumed from" in out
    a = [json.loads(l) for l in open(tmp_path / "a.jsonl")]
    b = [json.loads(l) for l in open(tmp_path / "b.jsonl")]
    assert len(a) == len(b) == 12
    for ra, rb in zip(a, b):
        assert ra["round"] == rb["round"]
        assert ra["accuracy"] == rb["accuracy"] and ra["f1"] == rb["f1"]


def test_data_plane_env_switch(monkeypatch):
    """FEDMI_DATA_PLANE selects the GPU FedAvg data plane of backend='auto' (CPU stays gloo)."""
    from fedmi.parallel.comm import resolve_backend
    monkeypatch.delenv("FEDMI_DATA_PLANE", raising=False)
    assert resolve_backend("auto", "cuda") == "xgmi"
    assert resolve_backend("auto", "cpu") == "gloo"
    for plane in ("rccl", "xgmi", "nccl"):
        monkeypatch.setenv("FEDMI_DATA_PLANE", plane.upper())
        assert resolve_backend("auto", "cuda") == plane
        assert resolve_backend("auto", "cpu") == "gloo"
    assert resolve_backend("gloo", "cpu") == "gloo"     # explicit choices are kept
    monkeypatch.setenv("FEDMI_DATA_PLANE", "tcp")
    import pytest
    with pytest.raises(ValueError):
        resolve_backend("auto", "cuda")
