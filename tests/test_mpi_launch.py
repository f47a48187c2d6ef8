"""Launch like the reference (``mpiexec -n k python <script>``): the processes
learn rank / size / local rank from the MPI launcher's environment (Open MPI, MPICH/Hydra).  No MPI launcher exists in this image, so the test starts the processes itself
with the environment Open MPI's and MPICH's launchers set."""
import os
import socket
import subprocess
import sys

import pytest

from fedmi.parallel.comm import launch_env

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(REPO, "FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py")
DATA = os.path.join(REPO, "data", "balanced_income_data.csv")
ALL_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE",
            "OMPI_COMM_WORLD_LOCAL_RANK", "PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID", "PMIX_RANK", "PMIX_SIZE",
            "PMIX_LOCAL_RANK", "SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID")


def _clean_env():
    return {k: v for k, v in os.environ.items() if k not in ALL_VARS}


def test_launch_env_recognises_launchers(monkeypatch):
    for k in ALL_VARS:
        monkeypatch.delenv(k, raising=False)
    assert launch_env() == (0, 1, 0, None)
    monkeypatch.setenv("PMI_RANK", "3")
    monkeypatch.setenv("PMI_SIZE", "4")
    assert launch_env() == (3, 4, 3, "mpich")
    monkeypatch.setenv("MPI_LOCALRANKID", "1")
    assert launch_env() == (3, 4, 1, "mpich")
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "2")
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "8")
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_RANK", "2")
    assert launch_env() == (2, 8, 2, "openmpi")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert launch_env()[3] == "torchrun"      # torchrun's variables win
    monkeypatch.setenv("WORLD_SIZE", "")
    assert launch_env()[3] == "openmpi"       # an empty variable does not count
    for k in ALL_VARS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("SLURM_PROCID", "0")
    monkeypatch.setenv("SLURM_NTASKS", "8")   # allocation-wide: a process started alone stays alone
    assert launch_env() == (0, 1, 0, None)


@pytest.mark.parametrize("flavour", ["openmpi", "mpich"])
def test_reference_entrypoint_under_mpi_environment(flavour):
    """Two CPU clients of the [C] entrypoint (BASELINE config 1) started the way mpiexec starts
    them: same command line, rank and size only in the launcher's variables."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = _clean_env()
        env.update(PYTHONPATH=REPO, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if flavour == "openmpi":
            env.update(OMPI_COMM_WORLD_RANK=str(r), OMPI_COMM_WORLD_SIZE="2", OMPI_COMM_WORLD_LOCAL_RANK=str(r))
        else:
            env.update(PMI_RANK=str(r), PMI_SIZE="2")
        cmd = [sys.executable, ENTRY, "--device", "cpu", "--backend", "gloo", "--engine", "torch", "--data", DATA,
               "--rounds", "3"]
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        assert p.returncode == 0, out
    # rank 0 reports both clients' metrics and the global ones, as the reference does
    assert "RANK 1 - Local Metrics (Round 3)" in outs[0] and "Global Metrics (Round 3)" in outs[0], outs[0]
