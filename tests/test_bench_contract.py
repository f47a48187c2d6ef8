"""bench.py contract: one JSON line with the required keys, for the headline [C] config, the
wide config (BASELINE config 3) and the packed sweep (BASELINE config 5), on one GPU with a
short run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(args, n=1, timeout=300):
    r = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["n_gpus"] == n and rec["value"] > 0 and rec["ms_per_step"] > 0
    return rec


def test_reference_chunking():
    """bench.py's shards follow the reference's _split_data chunking (C:57-60): 8000 // N rows per
    client, the last rank takes the remainder -- BASELINE.md's k-columns' shard sizes."""
    sys.path.insert(0, ROOT)
    from bench import REF_TRAIN_ROWS, reference_rows
    assert REF_TRAIN_ROWS == 8000
    for n, rows in ((1, 8000), (2, 4000), (4, 2000), (8, 1000)):
        assert [reference_rows(8000, n, r) for r in range(n)] == [rows] * n
    assert [reference_rows(8000, 3, r) for r in range(3)] == [2666, 2666, 2668]
    assert sum(reference_rows(10, 4, r) for r in range(4)) == 10


def _check_headline_config(rec, n):
    c = rec["config"]
    assert c["rows_per_client"] == 8000 // n and c["global_batch"] == 8000
    assert rec["scaling"] == "strong"
    assert c["early_stop"]["enabled"] is True and c["early_stop"]["patience"] > rec["steps"] + rec["warmup"]
    weak = rec["weak_8000_rows_per_client"]
    assert weak["rows_per_client"] == 8000 and weak["value"] > 0


@pytest.mark.gpu
def test_bench_headline_contract():
    rec = _run(["--steps", "50", "--warmup", "10", "--no-convergence"])
    assert rec["steps"] == 50 and rec["warmup"] == 10 and rec["dtype"] == "bf16"
    assert rec["vs_baseline"] > 0 and rec["replicas_consistent"] is True
    _check_headline_config(rec, 1)


@pytest.mark.gpu
def test_bench_self_launch_shared_gpu():
    """--gpus 2 without torchrun: bench.py starts 2 ranks itself (on one GPU with --share-gpu);
    the N > 1 round (lagged evaluation, FedAvg inside the Adam kernel over the peer protocol)
    runs and rank 0 alone prints the JSON line."""
    rec = _run(["--gpus", "2", "--share-gpu", "--steps", "40", "--warmup", "5", "--no-convergence",
                "--no-anchor"], n=2)
    assert rec["config"]["data_plane"] == "xgmi-oneshot+adam", rec["config"]
    assert rec["config"]["share_gpu"] is True
    assert rec["replicas_consistent"] is True
    _check_headline_config(rec, 2)
    assert rec["weak_8000_rows_per_client"]["replicas_consistent"] is True
    # per-kernel trace of the timed design; the other peer-plane designs timed the same way
    tr = rec["kernel_trace_us"]
    assert tr["launches"]["train"] == tr["launches"]["adam"] == tr["rounds"] and tr["train"] > 0
    pc = rec["plane_companions"]
    assert pc["ll_pull"]["round_design"] == "lagged-eval+adam-fedavg"
    assert pc["ll_pull"]["env"] == {"FEDMI_PEER_LL": "0"} and pc["ll_pull"]["exchange"] == "pull"
    assert pc["rsag"]["exchange"] == "rsag" and rec["config"]["exchange"] == "ll"
    assert pc["classic"]["round_design"] == "classic" and pc["classic"]["data_plane"] == "xgmi-oneshot"
    assert all(v["replicas_consistent"] is True and v["us_per_round"] > 0 for v in pc.values())


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_self_launch_eight_ranks_shared_gpu():
    """--gpus 8 (a whole MI355X node's world) with every rank on cuda:0: 8 self-launched ranks,
    the peer protocol's start-up self-test at world 8, and SCALE's own N = 8 round design -- lagged
    evaluation with FedAvg inside the Adam kernel -- on the bounded Adam grid that lets 8 ranks'
    exchanging blocks share one GPU (peer.shared_adam_grid), and the replica check on every rank."""
    rec = _run(["--gpus", "8", "--share-gpu", "--steps", "40", "--warmup", "5", "--no-convergence",
                "--no-anchor", "--no-plane-companions"], n=8, timeout=540)
    assert rec["config"]["data_plane"] == "xgmi-oneshot+adam", rec["config"]
    assert rec["config"]["round_design"] == "lagged-eval+adam-fedavg"
    assert rec["config"]["adam_grid"] == 16
    # 1000-row shards (63 workgroups of 16 rows): the lagged scoring runs on workgroups of its own
    assert rec["config"]["split_score"] is True
    assert rec["replicas_consistent"] is True
    _check_headline_config(rec, 8)


@pytest.mark.gpu
def test_bench_wide_contract():
    rec = _run(["--config", "wide", "--steps", "2", "--warmup", "1", "--wide-rows", "2048"])
    assert rec["config"]["model"] == "MLP 14-4096-4096-4096-2"
    assert rec["tflops_per_client"] > 0


@pytest.mark.gpu
def test_bench_sweep_contract():
    """BASELINE config 5 under the bench contract: 12 packed trials per GPU, a step = one round
    of every trial (three trial batches: one per hidden shape)."""
    rec = _run(["--config", "sweep", "--steps", "32", "--warmup", "16"])
    assert len(rec["config"]["trials"]) == 12 and "3 trial batches" in rec["config"]["parallelism"]
    assert rec["us_per_trial_round"] > 0 and 0.5 < rec["best_trial"]["train_acc_synthetic"] <= 1.0


def test_record_emitter_prints_once_and_watchdog_exits():
    """bench._Emitter: rank 0's record is printed exactly once -- after the N > 1 plane companions,
    or by the watchdog when they overrun, which names the extra that was running and ends the
    process with a NON-zero status (a hang must not pass for a clean run)."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "e = bench._Emitter({'value': 1.0}); e.emit(); e.emit(); "
            "w = bench._Emitter({'value': 2.0}); w.stage = 'plane_companions.ll_pull'; w.arm(0.3); "
            "time.sleep(20)") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert [x["value"] for x in lines] == [1.0, 2.0]
    assert "plane_companions.ll_pull" in lines[1]["plane_companions"]["error"]
    assert lines[1]["watchdog"] == {"fired": True, "stage": "plane_companions.ll_pull"}
    assert "watchdog fired during plane_companions.ll_pull" in p.stderr


@pytest.mark.parametrize("stage", ["rounds_to_target", "weak_8000_rows_per_client", "fp32_us_per_round",
                                   "torch_eager_us_per_round_1client"])
def test_watchdog_names_the_running_extra(stage):
    """A watchdog that fires during an untimed extra (every one runs after the headline record
    exists) files the error under that extra's own field, not as a plane-companion error."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "w = bench._Emitter({'value': 2.0, %r: None}); w.stage = %r; "
            "w.arm(0.3); time.sleep(20)") % (ROOT, stage, stage)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3
    rec = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")][0]
    assert stage in rec[stage]["error"] and rec["value"] == 2.0
    assert "plane_companions" not in rec
