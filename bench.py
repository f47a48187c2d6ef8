"""Flagship benchmark: federated rounds of the reference [C] workload on MI355X.

One process per GPU, each GPU one federated client (the reference's mpiexec ranks).  A
*step* is one full federated round exactly as the reference runs it
(``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:130-201``): a full-batch
forward/backward + Adam step + StepLR step on the client's shard (MLP 14->50->200->2,
bf16 MFMA operands with fp32 accumulation and fp32 master weights / Adam state by default, --dtype fp32 for exact-fp32 kernels), local evaluation of the post-step model on the shard (forward + argmax + weighted
metrics), and the sample-size-weighted FedAvg of all clients' weights.  At N > 1 the default
data plane is the xGMI exchange inside the Adam kernel (every parameter block pushes its
weighted update into every peer's LL ring over the direct links and sums its own ring in rank
order; the per-round metric tails ride the same exchange), RCCL the fallback.

Data: synthetic balanced-income-shaped rows (14 features, 2 classes) generated on the
device, weights random-init.  Shards follow the reference's chunking of its 8000 training
rows over the k clients (``_split_data``, FL_CustomMLP...Multiple_Rounds.py:57-60: chunk =
8000 // k, the last rank takes the remainder), i.e. 8000 / 4000 / 2000 / 1000 rows per
client at k = 1 / 2 / 4 / 8 -- exactly the shard sizes BASELINE.md's k-columns were measured
on, so the total work is fixed as N grows (strong scaling).  ``value`` = training samples
processed per second summed over all clients; ``vs_baseline`` divides by the reference's
measured train samples/s/client at the same k times N (408k / 398k / 323k /
264k; the reference's time excludes its eval and FedAvg, ours includes them).  The
early-stop rule (C:181-192, atol 1e-4 on the 4-metric vector) is evaluated on the device in
every timed round, with a patience no timed round can exhaust, so every timed round is live.
Companion key ``weak_8000_rows_per_client``: the same round with 8000 rows on every client
(per-GPU work fixed).  After the timed region, rounds-to-target on the real income CSV
(compat mode, this client count, the same shards) is measured and reported as
``rounds_to_target``.

    python bench.py --gpus 1 --steps 2000 --warmup 200
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 ...
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_PER_CLIENT = {1: 408e3, 2: 398e3, 4: 323e3, 8: 264e3}  # BASELINE.md, [C] train samples/s/client
METRIC = "samples/sec/client + rounds-to-target-accuracy, MLP on income data at 1/2/4/8 clients"


def ref_per_client(n: int) -> float:
    if n in REF_PER_CLIENT:
        return REF_PER_CLIENT[n]
    ks = sorted(REF_PER_CLIENT)
    k = min(ks, key=lambda x: abs(x - n))
    return REF_PER_CLIENT[k]


REF_TRAIN_ROWS = 8000  # the reference's training split (8000 of 10 000 rows, C:239)


def reference_rows(total: int, world: int, rank: int) -> int:
    """Rows of ``rank``'s shard under the reference's chunking (C:57-60): chunk = max(1, total //
    world) rows per rank, the last rank also takes the remainder."""
    chunk = max(1, total // world)
    if rank < world - 1:
        return chunk
    return total - chunk * (world - 1)


def synth_shard(n_rows: int, rank: int, device, seed: int = 7):
    """Income-shaped rows generated on the device by the Philox kernel."""
    from fedmi.data.synthetic import device_shard
    return device_shard(n_rows, rank, device, seed)


def rounds_to_target(comm, targets=(0.80, 0.83), max_rounds=300, dtype="fp32", lagged_eval=True):
    """Reference-compat convergence on the real CSV at this client count (untimed)."""
    from fedmi.data.tabular import load_tabular
    from fedmi.fl.engine import EngineConfig
    from fedmi.fl.trainer import FederatedMLPLearning
    ds = load_tabular()
    cfg = EngineConfig(max_rounds=max_rounds, graph_rounds=16, dtype=dtype, lagged_eval=lagged_eval)
    tr = FederatedMLPLearning(ds.X_train, ds.y_train, comm.rank, comm.size, comm=comm, config=cfg,
                              mode="compat", seed=0)
    tr.train_and_evaluate(comm, rounds=max_rounds, verbose=False)
    h = tr.history()
    acc = h["global"][:, 0]
    out = {}
    for t in targets:
        hit = np.flatnonzero(acc >= t)
        out[f"{t:.2f}"] = int(hit[0]) + 1 if len(hit) else None
    out["early_stop_round"] = int(h["stop_round"]) if h["stop_round"] >= 0 else None
    out["final_acc"] = float(acc[-1]) if len(acc) else None
    out["dtype"] = dtype
    return out


_T_START = time.perf_counter()


def _progress(msg: str) -> None:
    """FEDMI_BENCH_PROGRESS=1: stage markers with elapsed seconds on stderr (long shared-GPU runs)."""
    if os.environ.get("FEDMI_BENCH_PROGRESS") == "1":
        print(f"[bench {os.environ.get('RANK', '0')} +{time.perf_counter() - _T_START:.1f}s] {msg}",
              file=sys.stderr, flush=True)


def _self_launch(a, argv) -> int:
    """``--gpus N`` (N > 1) without a torch.distributed environment: start N ranks with
    torch.distributed.run as a CHILD process (this process never touches the GPU) and exit
    with its code.  Only rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    # build (or verify) the extension ONCE here -- compilation never touches the GPU -- so the N
    # ranks do not all find it missing / stale and compile it at the same time
    from fedmi.ops import build as _b
    _b.build()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__),
           *(sys.argv[1:] if argv is None else list(argv))]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _pick_graph_rounds(steps: int, cap: int = 64) -> int:
    """Largest even g <= cap dividing the timed steps (so the timed region is whole graph
    replays); 2 if none does."""
    for g in range(min(cap, steps) & ~1, 1, -2):
        if steps % g == 0:
            return g
    return 2


def torch_eager_anchor(X, y, dims, rounds: int = 60, warmup: int = 10) -> float:
    """Same-box anchor: the reference's round (eager torch nn.Linear / CrossEntropyLoss /
    Adam / StepLR on the GPU, get/set weights through the host, C:63-120) for ONE client on
    this GPU, microseconds per round."""
    from fedmi.fl.engine import EngineConfig, TorchRoundEngine
    from fedmi.models.mlp import init_flat
    cfg = EngineConfig(hidden=tuple(dims[1:-1]), max_rounds=rounds + warmup + 2, early_stop=False)
    eng = TorchRoundEngine(X.cpu().numpy(), y.cpu().numpy().astype(np.int64), dims[-1], cfg, None,
                           init_flat(dims, seed=0), device=X.device)
    eng.run(warmup)
    torch.cuda.synchronize(X.device)
    t0 = time.perf_counter()
    eng.run(rounds)
    torch.cuda.synchronize(X.device)
    return (time.perf_counter() - t0) / rounds * 1e6


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--rows-per-client", type=int, default=0,
                    help="rows on every client (0: the reference's chunking of --total-rows over the N clients, "
                         "C:57-60 -- 8000 // N each, the last rank takes the remainder)")
    ap.add_argument("--total-rows", type=int, default=REF_TRAIN_ROWS)
    ap.add_argument("--no-weak", action="store_true",
                    help="skip the companion run with 8000 rows on every client (weak scaling)")
    ap.add_argument("--no-early-stop", dest="early_stop", action="store_false",
                    help="do not evaluate the early-stop rule in the timed rounds")
    ap.add_argument("--patience", type=int, default=0,
                    help="early-stop patience in the timed run (0: longer than the run, so every timed round is live)")
    ap.add_argument("--hidden", type=int, nargs="+", default=[50, 200])
    ap.add_argument("--rows-per-block", type=int, default=0,
                    help="rows per workgroup of the fused kernels (0: the engine's choice for the shard size)")
    ap.add_argument("--graph-rounds", type=int, default=0,
                    help="rounds per captured HIP graph (0: largest even divisor of --steps up to 64)")
    ap.add_argument("--backend", default="auto", choices=["auto", "xgmi", "rccl", "nccl"],
                    help="FedAvg data plane: one-shot xGMI peer all-reduce (falls back to RCCL) | RCCL | torch nccl "
                         "(auto: $FEDMI_DATA_PLANE, default xgmi)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="debug: every rank on cuda:0 (xGMI peer protocol between processes of one GPU, no RCCL), "
                         "so the N > 1 path runs on a one-GPU box")
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16"],
                    help="MFMA operand type of the fused kernels (fp32 accumulate, fp32 master weights)")
    ap.add_argument("--prime-replays", type=int, default=1,
                    help="untimed replays of the timed region's graph after its capture (warm-up; 1 / 2 / 3 "
                         "measured the same at 20 steps, profiles/prime_replays_ab_r5.log)")
    ap.add_argument("--trace-rounds", type=int, default=8,
                    help="after the timed region (untimed): this many rounds of the same round design issued "
                         "eagerly with a hipEvent per launch (HipRoundEngine.trace) -> per-kernel us per round in "
                         "the record's kernel_trace_us (0: off)")
    ap.add_argument("--no-plane-companions", action="store_true",
                    help="N > 1 on the xGMI plane: skip the untimed-for-the-headline companions that time the same "
                         "shard with the pull protocol (FEDMI_PEER_LL=0) and with classic rounds (lagged_eval off)")
    ap.add_argument("--companion-timeout", type=float, default=300.0,
                    help="seconds the untimed extras (the weak-scaling companion, the eager anchor, the fp32 round, "
                         "rounds-to-target, the N > 1 plane companions) may take before a watchdog prints the "
                         "headline record and exits with status 3")
    ap.add_argument("--no-convergence", action="store_true")
    ap.add_argument("--no-anchor", action="store_true", help="skip the same-box eager torch anchor")
    ap.add_argument("--no-fp32", action="store_true", help="skip the untimed fp32-kernel round (one client)")
    ap.add_argument("--config", default="c", choices=["c", "wide", "sweep"],
                    help="c: the reference [C] workload (default, the headline metric) | wide: BASELINE config 3, "
                         "MLP 14-4096-4096-4096-2 on --wide-rows synthetic rows per client, bf16 NT GEMMs, "
                         "per-layer FedAvg buckets over RCCL | sweep: BASELINE config 5, --trials FedAvg trials "
                         "({hidden} x {lr} x {local steps} grid) packed per GPU, a step = one round of every trial")
    ap.add_argument("--trials", type=int, default=12, help="--config sweep: trials per GPU (first K of the grid)")
    ap.add_argument("--trial-rows-per-block", type=int, default=-1,
                    help="--config sweep: rows per workgroup of the trial batches (-1: the largest that fits LDS, "
                         "64 first; 0: the single-engine choice, 32)")
    ap.add_argument("--wide-rows", type=int, default=131072,
                    help="rows per client (BASELINE config 3 names 1e8-row shards: 12500000 per client at k = 8)")
    ap.add_argument("--micro-batch", type=int, default=131072, help="--config wide: rows per micro-batch")
    ap.add_argument("--wide-allreduce", default="fp32", choices=["fp32", "bf16"],
                    help="--config wide: FedAvg bucket dtype on the wire (bf16: the round's delta; fp32 master "
                         "weights either way)")
    ap.add_argument("--no-fused-eval", dest="fused_eval", action="store_false",
                    help="--config wide: evaluate every round with its own forward pass over the shard (the round "
                         "shape of a client at N > 1, where the next round's forward sees the global model) even "
                         "at one client")
    ap.add_argument("--wide-lr", type=float, default=None,
                    help="--config wide: Adam lr (default fedmi.fl.wide.WIDE_LR = 1e-4; 0.004 diverges at width 4096)")
    a = ap.parse_args(argv)
    from fedmi.parallel.comm import launch_env
    if a.gpus > 1 and launch_env()[1] == 1:  # no multi-process launcher around us: start the ranks
        return _self_launch(a, argv)
    if a.config == "wide":
        return main_wide(a)
    if a.config == "sweep":
        return main_sweep(a)

    from fedmi.fl.engine import EngineConfig, HipRoundEngine
    from fedmi.models.mlp import init_flat
    from fedmi.parallel.comm import get_world
    import torch.distributed as dist

    from fedmi.parallel.comm import resolve_backend
    a.backend = resolve_backend(a.backend, "cuda")
    if a.share_gpu:
        if a.backend != "xgmi":
            raise SystemExit("--share-gpu runs the xGMI peer protocol (RCCL cannot put two ranks on one GPU)")
        comm = get_world(backend="xgmi", device="cuda:0", rccl=False)
    else:
        comm = get_world(backend=a.backend, device="cuda")
    N = comm.size
    if N != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={N}")
    dev = comm.device
    dims = [14, *a.hidden, 2]
    g = a.graph_rounds or _pick_graph_rounds(a.steps)
    # (ranks sharing one GPU: the Adam kernels' in-kernel chunk exchange needs every rank's
    # exchanging blocks resident at once; make_peer_allreduce bounds the grid for that --
    # fedmi.parallel.peer.shared_adam_grid -- so the N > 1 round design is the same as on N GPUs)
    trace_warm = 2  # untraced rounds behind the trace's gate (absorb the ranks' start skew)
    max_rounds = a.warmup + a.steps + max(1, a.prime_replays) * g + 16 + max(0, a.trace_rounds) + trace_warm
    # the early-stop rule runs in every round; a patience above the run's length keeps every
    # timed round live (a stop would turn the remaining rounds into no-ops)
    patience = a.patience if a.patience > 0 else max_rounds + 1
    if patience <= max_rounds and a.early_stop:
        print(f"warning: patience {patience} may stop the timed region early", file=sys.stderr)

    def barrier():
        if N > 1:
            dist.barrier()

    # every engine of this process issues on ONE stream (HipRoundEngine `stream`: with ranks sharing
    # a GPU, the companion run's engine on a fresh stream ran 2.3x slower)
    stream = torch.cuda.Stream(device=dev)

    def timed_rounds(rows_local: int, rows_total: int, dtype: str = a.dtype, trace: int = 0, lagged_eval: bool = True):
        """Build a client with `rows_local` rows (FedAvg weight rows_local / rows_total), warm up,
        time exactly a.steps rounds (max over ranks), then (untimed) trace `trace` rounds, close +
        check; returns (dt, engine, primed, trace record or None)."""
        _progress(f"engine: {rows_local} rows, {dtype}, lagged_eval={lagged_eval}")
        X, y = synth_shard(rows_local, comm.rank, dev)
        cfg = EngineConfig(hidden=tuple(a.hidden), max_rounds=max_rounds, early_stop=a.early_stop,
                           patience=patience, rows_per_block=a.rows_per_block, graph_rounds=g,
                           dtype=dtype, lagged_eval=lagged_eval)
        eng = HipRoundEngine(X, y, 2, cfg, comm, init_flat(dims, seed=comm.rank), n_total=rows_total, stream=stream)
        # warm-up: the requested rounds, then (uncounted) the graph of the timed region is
        # captured, instantiated and replayed once, so the timed steps are steady-state replays
        _progress(f"warm-up ({eng.aggregation})")
        eng.run(a.warmup, check_every=max(a.warmup, 1))
        # host plane (peer set-up and RCCL both unavailable): rounds are aggregated from Python,
        # eagerly -- slower, but the run still yields a number labelled data_plane 'host'
        primed = eng.prime_graph(g, replays=a.prime_replays) if eng._engine_reduces() or N == 1 else 0
        _progress("timed region")
        eng.stream.synchronize()
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        eng._issue(a.steps, close=False)  # exactly K rounds, no host polling inside
        torch.cuda.synchronize(dev)       # (waits for the engine's stream too: one wake-up, not two)
        barrier()
        dt = time.perf_counter() - t0
        eng._check_peer()  # a failure reported on the xGMI plane: no number for these rounds
        if N > 1:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        tr, traced = None, 0
        if trace > 0 and (eng._engine_reduces() or N == 1):
            # per-kernel breakdown of the same round design (eager, events per launch); the max
            # over ranks of each kind (at N > 1 waiting for a slower rank lands in "adam")
            barrier()
            _progress("trace")
            tr = eng.trace(trace, close=False, warm=trace_warm)
            traced = trace + trace_warm
            kinds = sorted(k for k, v in tr.items() if isinstance(v, float))
            if N > 1:
                t = torch.tensor([tr[k] for k in kinds], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                tr.update(zip(kinds, t.tolist()))
            tr = {**{k: round(tr[k], 3) for k in kinds}, "launches": tr["launches"], "rounds": tr["rounds"],
                  "method": "eager rounds behind a gate kernel, hipEvent after every launch (each interval "
                            "carries ~1.5 us of eager launch + marker cost over the kernel's rocprofv3 duration, "
                            "profiles/kernel_trace_r5.log); max over ranks"}
        eng._issue(1)  # untimed closing round: scores the last timed (or traced) round
        eng.sync_history()
        h = eng.history()
        # every timed round was live and folded (a stop would leave rounds_run short)
        assert h["rounds_run"] == a.warmup + primed + a.steps + traced + 1 and h["stop_round"] < 0, \
            (h["rounds_run"], primed, h["stop_round"])
        return dt, eng, primed, tr

    rows_local = a.rows_per_client or reference_rows(a.total_rows, N, comm.rank)
    rows_total = a.rows_per_client * N if a.rows_per_client else a.total_rows
    from fedmi.parallel.peer import PeerFailure
    plane_failure = None
    try:
        dt, eng, primed, ktrace = timed_rounds(rows_local, rows_total, trace=max(0, a.trace_rounds))
    except PeerFailure as e:
        # The xGMI plane reported a failure (a wait timed out): every rank's failure word is set,
        # so every rank lands here together.  Re-run the timed rounds on the next data plane (RCCL,
        # else the host) and label the record, instead of ending the run without a number.
        if N == 1:
            raise
        plane_failure = str(e)[:300]
        print(f"[bench] rank {comm.rank}: {plane_failure}; re-running the timed rounds without the xGMI plane",
              file=sys.stderr, flush=True)
        comm.peer_allreduce = False
        gc.collect()
        dt, eng, primed, ktrace = timed_rounds(rows_local, rows_total, trace=max(0, a.trace_rounds))
    h = eng.history()
    # every rank must hold the same global model and metric history (raises otherwise: no number
    # is reported for a run whose FedAvg was not FedAvg)
    from fedmi.parallel.consistency import check_replicas
    replicas_ok = check_replicas(comm, [eng.global_flat(), np.asarray(h["global"])])
    value = rows_total * a.steps / dt
    # what the record needs from the timed engine; then it is released (its graph, buffers and
    # xGMI peer mappings) before any other engine of this process runs
    def round_design(e) -> str:
        return ("fused-eval" if N == 1 else
                "lagged-eval+adam-fedavg" if e.engine.adam_exchange else
                "lagged-eval+late-fold" if e.engine.late_fold else
                "lagged-eval" if e.engine.lagged else "classic")

    def exchange(e) -> str:
        """Weight-chunk protocol of the Adam-fused exchange: 'll' (every rank pushes every value to
        every rank), 'rsag' (reduce-scatter + all-gather on the LL ring), 'pull' (publish / wait /
        pull); 'none' without an in-kernel exchange."""
        if e._peer is None or not e.engine.adam_exchange:
            return "none"
        return "rsag" if e._peer.uses_rsag else ("ll" if e._peer.uses_ll else "pull")

    design = {"aggregation": eng.aggregation, "exchange": exchange(eng),
              "round_design": round_design(eng),
              "rows_per_block": eng.R, "plain_fwd": bool(eng.layout.get("plain_fwd", False)),
              "split_score": bool(eng.layout.get("split_score", False)),
              "adam_grid": int(eng._peer.adam_grid) if eng._peer is not None else 0,
              "peer_timeout_s": float(eng._peer.timeout_s) if eng._peer is not None else None,
              "lagged_eval": eng.cfg.lagged_eval, "final_acc": float(h["global"][-1][0])}
    X, y = eng.X, eng.y
    del eng
    gc.collect()
    torch.cuda.synchronize(dev)
    rec = None
    if comm.rank == 0:
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "train samples/s (sum over clients; step = 1 federated round incl. eval + FedAvg)",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if a.rows_per_client else "strong",
            "vs_baseline": value / (ref_per_client(N) * N),
            "dtype": a.dtype,
            "data": (f"synthetic income-shaped (device Philox), {rows_total} training rows "
                     + (f"({a.rows_per_client}/client)" if a.rows_per_client else
                        f"chunked over {N} client(s) as the reference does ({rows_local} on rank {comm.rank})")
                     + "; random-init weights"),
            "config": {"model": f"MLP {'-'.join(map(str, dims))} (reference [C])",
                       "global_batch": rows_total, "seq_len": 1,
                       "parallelism": f"fedavg{N} (1 client/{'shared ' if a.share_gpu else ''}GPU, "
                                      f"{design['aggregation']} all-reduce)",
                       "data_plane": design["aggregation"],
                       "adam_grid": design["adam_grid"],
                       "round_design": design["round_design"],
                       "exchange": design["exchange"],
                       "rccl_env": comm.rccl_env,
                       "peer_timeout_s": design["peer_timeout_s"],
                       "rows_per_client": a.rows_per_client or reference_rows(a.total_rows, N, 0),
                       "rows_last_client": a.rows_per_client or reference_rows(a.total_rows, N, N - 1),
                       "rows_per_block": design["rows_per_block"],
                       "optimizer": "Adam(0.004)+StepLR(30,0.5)",
                       "early_stop": {"enabled": bool(a.early_stop), "patience": patience, "atol": 1e-4,
                                      "rtol": 1e-5, "note": "rule evaluated on the device every timed round; "
                                      "patience longer than the run so every timed round is live"},
                       "plain_fwd": design["plain_fwd"], "split_score": design["split_score"],
                       "graph_rounds": g, "share_gpu": bool(a.share_gpu)},
            "samples_per_sec_per_client": value / N,
            "us_per_round": dt / a.steps * 1e6,
            "kernel_trace_us": ktrace,
            "plane_companions": None,
            "weak_8000_rows_per_client": None,
            "torch_eager_us_per_round_1client": None,
            "fp32_us_per_round": None if a.dtype != "fp32" else dt / a.steps * 1e6,
            "final_train_acc_synthetic": design["final_acc"],
            "replicas_consistent": replicas_ok,
            "rounds_to_target": None,
        }
        if plane_failure is not None:
            rec["data_plane_failure"] = plane_failure
        if N > 1 and design["aggregation"] == "host":
            rec["warning"] = ("FedAvg went through the HOST plane (gloo all-gather, rank-order sums): the xGMI "
                              "peer set-up and the RCCL bootstrap were both unavailable; this is not the device "
                              "data plane's number")
    # The untimed extras run under a watchdog once the headline record exists: rank 0 prints it
    # exactly once whatever happens to them (an extra that raises is recorded; one stuck in a
    # collective or a peer wait ends the process when the budget runs out) -- the weak-scaling
    # companion, the eager anchor and the fp32 round included, so no extra can cost the headline.
    emit = _Emitter(rec)
    emit.arm(a.companion_timeout)
    # companion: per-GPU work fixed at the reference's one-client shard (8000 rows on every client)
    emit.stage = "weak_8000_rows_per_client"
    weak = None
    if not a.rows_per_client and not a.no_weak:
        if N == 1 and rows_local == REF_TRAIN_ROWS:
            weak = {"value": value, "us_per_round": dt / a.steps * 1e6, "rows_per_client": REF_TRAIN_ROWS}
        else:
            try:
                dtw, engw, _, _ = timed_rounds(REF_TRAIN_ROWS, REF_TRAIN_ROWS * N)
                weak = {"value": REF_TRAIN_ROWS * N * a.steps / dtw, "us_per_round": dtw / a.steps * 1e6,
                        "rows_per_client": REF_TRAIN_ROWS, "scaling": "weak",
                        "replicas_consistent": check_replicas(comm, [engw.global_flat()])}
                del engw
            except Exception as e:  # noqa: BLE001 -- recorded; a PeerFailure is raised on every rank together
                weak = {"error": f"{type(e).__name__}: {e}"[:400]}
            gc.collect()
    if rec is not None:
        rec["weak_8000_rows_per_client"] = weak
    if not a.no_anchor:
        emit.stage = "torch_eager_us_per_round_1client"
        if comm.rank == 0:
            try:
                rec["torch_eager_us_per_round_1client"] = torch_eager_anchor(X, y, dims)
            except Exception as e:  # noqa: BLE001
                rec["torch_eager_us_per_round_1client"] = {"error": f"{type(e).__name__}: {e}"[:400]}
        barrier()
    if N == 1 and a.dtype != "fp32" and not a.no_fp32:
        # the reference-precision companion, timed EXACTLY like the headline: same shard, same
        # --warmup / --steps, early-stop rule live, one graph replay of the timed steps
        emit.stage = "fp32_us_per_round"
        try:
            dtf, engf, _, _ = timed_rounds(rows_local, rows_total, dtype="fp32")
            if rec is not None:
                rec["fp32_us_per_round"] = dtf / a.steps * 1e6
            del engf
        except Exception as e:  # noqa: BLE001 -- one client: nothing collective to leave behind
            if rec is not None:
                rec["fp32_us_per_round"] = {"error": f"{type(e).__name__}: {e}"[:400]}
        gc.collect()
    if not a.no_convergence:
        emit.stage = "rounds_to_target"
        ok = True
        try:
            # rounds-to-target is measured with the same kernels (dtype) as the throughput
            rtt = rounds_to_target(comm, dtype=a.dtype, lagged_eval=design["lagged_eval"])
            if rec is not None:
                rec["rounds_to_target"] = rtt
        except Exception as e:  # noqa: BLE001
            ok = False
            if rec is not None:
                rec["rounds_to_target"] = {"error": f"{type(e).__name__}: {e}"[:400]}
        # every rank learns whether rounds-to-target failed anywhere: a rank that raised must not
        # leave the others to enter the collective companions alone
        if N > 1:
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = bool(t.item())
        if not ok:
            if rec is not None and "error" not in (rec.get("rounds_to_target") or {}):
                rec["rounds_to_target"] = {"error": "failed on another rank"}
            emit.emit()
    # N > 1 on the xGMI plane: the same shard timed exactly like the headline with the other round
    # designs the peer plane offers -- data for choosing between them on real xGMI links, which no
    # one-GPU session can measure (each companion is its own engine)
    if N > 1 and design["aggregation"].startswith("xgmi") and not a.no_plane_companions and not emit.done:
        planes = {}
        try:
            for name, env, lagged in (("ll_pull", {"FEDMI_PEER_LL": "0"}, True),
                                      ("rsag", {"FEDMI_PEER_RSAG": "1"}, True),
                                      ("classic", {}, False)):
                emit.stage = f"plane_companions.{name}"
                old = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                try:
                    dtc, engc, _, trc = timed_rounds(rows_local, rows_total, trace=max(0, a.trace_rounds),
                                                     lagged_eval=lagged)
                    planes[name] = {"us_per_round": dtc / a.steps * 1e6, "value": rows_total * a.steps / dtc,
                                    "round_design": round_design(engc), "data_plane": engc.aggregation,
                                    "exchange": exchange(engc),
                                    "env": env, "kernel_trace_us": trc,
                                    "replicas_consistent": check_replicas(comm, [engc.global_flat()])}
                    del engc
                    gc.collect()
                finally:
                    for k, v in old.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
                if rec is not None:
                    rec["plane_companions"] = dict(planes)
        except Exception as e:  # noqa: BLE001 -- the headline stands; the companion's failure is recorded
            if rec is not None:
                rec["plane_companions"] = {**planes, "error": f"{type(e).__name__}: {e}"[:400]}
            emit.emit()
    emit.emit()
    comm.close()
    emit.disarm()
    return 0


WATCHDOG_EXIT = 3  # exit status of a run whose untimed extras overran (the record is still printed)


class _Emitter:
    """Rank 0's one JSON line, printed exactly once: normally after the untimed extras, or by a
    watchdog when they exceed their time budget -- then the record names the extra that was
    running (``stage``), and the process exits at once with status WATCHDOG_EXIT on every rank
    (an extra stuck in a collective or a peer wait must not cost the headline record, and must
    not pass for a clean run either)."""

    def __init__(self, rec):
        import threading
        self.rec, self.lock, self.done, self.timer = rec, threading.Lock(), False, None
        self.stage = None   # the untimed extra running now

    def emit(self) -> None:
        with self.lock:
            if not self.done and self.rec is not None:
                print(json.dumps(self.rec), flush=True)
            self.done = True

    def _expire(self) -> None:
        stage = self.stage or "untimed extras"
        with self.lock:
            if self.rec is not None and not self.done:
                msg = f"watchdog: {stage} exceeded the extras' time budget"
                # filed under the running extra's own field (the plane companions share one)
                key = stage.split(".")[0] if stage.split(".")[0] in self.rec else "plane_companions"
                prev = self.rec.get(key)
                self.rec[key] = {**(prev if isinstance(prev, dict) else {}), "error": msg}
                self.rec["watchdog"] = {"fired": True, "stage": stage}
        self.emit()
        print(f"[bench] rank {os.environ.get('RANK', '0')}: watchdog fired during {stage}", file=sys.stderr, flush=True)
        # release this rank's spinning device waits and tell the peers (xGMI plane), then exit
        if "fedmi.parallel.peer" in sys.modules:
            sys.modules["fedmi.parallel.peer"].abort_all()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(WATCHDOG_EXIT)

    def arm(self, seconds: float) -> None:
        import threading
        self.timer = threading.Timer(seconds, self._expire)
        self.timer.daemon = True
        self.timer.start()

    def disarm(self) -> None:
        if self.timer is not None:
            self.timer.cancel()


def main_wide(a) -> None:
    """BASELINE config 3 under the same contract: a step is one federated round of the wide
    client (full-batch local Adam step over the shard + per-layer FedAvg buckets)."""
    from fedmi.fl.wide import WIDE_LR, WideClient
    from fedmi.parallel.comm import get_world
    import torch.distributed as dist

    from fedmi.parallel.comm import resolve_backend
    a.backend = resolve_backend(a.backend, "cuda")
    comm = get_world(backend="rccl" if a.backend == "xgmi" else a.backend, device="cuda", rccl_proto="Simple")
    N = comm.size
    if N != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={N}")
    dims = [14, 4096, 4096, 4096, 2]
    X, y = synth_shard(a.wide_rows, comm.rank, comm.device)
    lr = a.wide_lr if a.wide_lr is not None else WIDE_LR
    c = WideClient(X, y, dims, comm=comm if N > 1 else None, n_total=a.wide_rows * N, dtype="bf16", seed=0,
                   micro_batch=a.micro_batch, allreduce_dtype=a.wide_allreduce, lr=lr,
                   fused_eval=None if a.fused_eval else False)

    def barrier():
        if N > 1:
            dist.barrier()

    # every round as the reference runs it: local step, local evaluation of the post-step model
    # on the whole shard (device-side confusion counts), FedAvg
    first_loss = None
    for i in range(a.warmup):
        c.run_round(evaluate=True)
        if i == 0:
            first_loss = c.loss()   # (untimed: warm-up) the loss of round 1's local step
    c.sync()
    torch.cuda.synchronize(comm.device)
    barrier()
    torch.cuda.synchronize(comm.device)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        c.run_round(evaluate=True)
    c.sync()
    torch.cuda.synchronize(comm.device)
    barrier()
    dt = time.perf_counter() - t0
    if N > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    value = a.wide_rows * N * a.steps / dt
    last_loss = c.loss()
    from fedmi.parallel.consistency import check_replicas
    replicas_ok = check_replicas(comm, [c.params])
    if comm.rank == 0:
        print(json.dumps({
            "metric": "train samples/s, wide-MLP FedAvg (BASELINE config 3)", "value": value,
            "unit": "train samples/s (sum over clients; step = 1 federated round: full-batch Adam step + local "
                    "evaluation of the shard + FedAvg)",
            "n_gpus": N, "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic income-shaped (device Philox), {a.wide_rows} rows/client; random-init weights",
            "config": {"model": "MLP " + "-".join(map(str, dims)), "global_batch": a.wide_rows * N, "seq_len": 1,
                       "parallelism": f"fedavg{N} (1 client/GPU, per-layer RCCL buckets, "
                                      f"{a.wide_allreduce} on the wire)", "rccl_env": comm.rccl_env},
            "tflops_per_client": c.flops_per_round / (dt / a.steps) / 1e12,
            # one client: round r's local evaluation is scored from round r+1's training forward
            # (same weights, rows and kernels: bit-identical counts), so tflops counts executed work
            "round_design": "fused-eval" if c.fused_eval else "separate-eval",
            "local_train_acc_synthetic": c.metrics()["accuracy"],
            "lr": lr, "rounds_run": c.round,
            "loss_first_round": first_loss, "loss_last_round": last_loss,
            "replicas_consistent": replicas_ok,
            "micro_batch": c.mb,
        }), flush=True)
    comm.close()


def main_sweep(a) -> int:
    """BASELINE config 5 under the same contract: every GPU (client) runs ``--trials`` FedAvg
    trials of the [C] workload at once -- hidden {(50,200),(100,50),(50,100)} x lr {0.002,0.004}
    x local steps {1,2} (fedmi.hpo.fed_sweep; same-shape trials as native trial batches, the
    whole K-trial round one HIP graph, one shared all-reduce for all trials).  A step is one
    round of every trial; ``value`` = trial-rounds/s summed over GPUs."""
    from fedmi.fl.engine import EngineConfig
    from fedmi.hpo.fed_sweep import FedTrialGroup, grid
    from fedmi.parallel.comm import get_world, resolve_backend
    import torch.distributed as dist

    a.backend = resolve_backend(a.backend, "cuda")
    comm = get_world(backend="rccl" if a.backend == "xgmi" else a.backend, device="cuda")
    N = comm.size
    if N != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={N}")
    trials = grid(((50, 200), (100, 50), (50, 100)), (0.002, 0.004), (1, 2))
    trials = (trials * ((a.trials + len(trials) - 1) // len(trials)))[:a.trials]
    # rows per client: --rows-per-client, else the reference's chunking of --total-rows (C:57-60)
    rows_local = a.rows_per_client or reference_rows(a.total_rows, N, comm.rank)
    rows_total = a.rows_per_client * N if a.rows_per_client else a.total_rows
    X, y = synth_shard(rows_local, comm.rank, comm.device)
    g_rounds = 16
    base = EngineConfig(max_rounds=a.warmup + a.steps + 2 * g_rounds + 4, early_stop=False, dtype=a.dtype,
                        rows_per_block=a.trial_rows_per_block,
                        graph_rounds=g_rounds)
    grp = FedTrialGroup(X, y, 2, trials, comm if N > 1 else None, base, n_total=rows_total,
                        group_graph_rounds=g_rounds)

    def barrier():
        if N > 1:
            dist.barrier()

    grp.run(max(a.warmup, g_rounds))   # includes the group graph's capture and first replay
    torch.cuda.synchronize(comm.device)
    barrier()
    torch.cuda.synchronize(comm.device)
    t0 = time.perf_counter()
    grp.run(a.steps)
    torch.cuda.synchronize(comm.device)
    barrier()
    dt = time.perf_counter() - t0
    if N > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    value = len(trials) * a.steps * N / dt
    from fedmi.parallel.consistency import check_replicas
    replicas_ok = check_replicas(comm, [e.global_flat() for e in grp.engines])
    best = grp.best()
    if comm.rank == 0:
        print(json.dumps({
            "metric": "trial-rounds/s, packed federated hyperparameter sweep (BASELINE config 5)", "value": value,
            "unit": "trial-rounds/s (sum over GPUs; step = one federated round of every trial incl. eval + FedAvg)",
            "n_gpus": N, "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak" if a.rows_per_client else "strong", "vs_baseline": None,
            "dtype": a.dtype,
            "data": f"synthetic income-shaped (device Philox), {rows_total} training rows ({rows_local} on rank 0); "
                    "random-init weights",
            "config": {"model": "MLP 14-{hidden}-2 grid", "global_batch": rows_total, "seq_len": 1,
                       "parallelism": f"fedavg{N} x {len(trials)} trials/GPU ({len(grp.batches)} trial batches, "
                                      f"one all-reduce per round)", "rccl_env": comm.rccl_env,
                       "trials": [[list(t.hidden), t.lr, t.local_steps] for t in trials],
                       "rows_per_block": {"x".join(map(str, t.hidden)): e.R for t, e in zip(trials, grp.engines)}},
            "us_per_trial_round": dt / (a.steps * len(trials)) * 1e6,
            "replicas_consistent": replicas_ok,
            "best_trial": {"hidden": list(best.hidden), "lr": best.lr, "local_steps": best.local_steps,
                           "train_acc_synthetic": best.final["accuracy"]},
        }), flush=True)
    comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
