"""[C] entrypoint flags of the north-star list: --clients (K simulated clients in
one process), --synthetic (income-shaped rows instead of the CSV), --local-epochs (alias of
--local-steps), on the CPU plumbing path."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = os.path.join(ROOT, "FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py")


def _run(args):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, C, "--device", "cpu", "--backend", "gloo", "--engine", "torch", *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_clients_simulates_a_federation(tmp_path):
    out = _run(["--clients", "4", "--rounds", "12", "--jsonl", str(tmp_path / "m.jsonl")])
    assert "4 simulated clients (torch): 12 rounds" in out
    assert "RANK 3 - Local Metrics (Round 12)" in out      # reference console format, every client
    rows = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert len(rows) == 12 and len(rows[-1]["per_rank"]) == 4 and rows[-1]["accuracy"] > 0.7


def test_synthetic_rows_and_local_epochs():
    out = _run(["--synthetic", "--synthetic-rows", "2000", "--rounds", "4", "--local-epochs", "2", "--mode", "correct"])
    assert "Global Metrics (Round 4)" in out
    assert "Held-out test metrics of the aggregated model" in out


def test_hpo_grid_json():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    H = os.path.join(ROOT, "hyperparameters_tuning.py")
    r = subprocess.run([sys.executable, H, "--device", "cpu", "--federated", "--rounds", "3", "--quiet", "--hpo-grid",
                        '{"hidden": [[20], [10, 5]], "lr": [0.004], "local_steps": [1, 2]}'],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "for 4 trials x 3 rounds" in r.stdout
