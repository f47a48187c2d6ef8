"""Entrypoint [C]: multi-round FedAvg of a custom MLP classifier (fedmi engine).

Same name and defaults as the reference script
(``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py``: MLP 14->50->200->2, Adam
0.004, StepLR(30, 0.5), 300 rounds, patience 10, atol 1e-4), defaulting to the shipped
``balanced_income_data.csv`` / ``income`` (the reference's hard-coded
diabetes CSV is not in the repo).

Launch (one process per GPU, each a federated client):

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 \
        FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py

or ``python FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py`` for one client.
``--device cpu --backend gloo`` reproduces the reference's CPU configuration.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from fedmi.ckpt.checkpoint import resume, save_checkpoint
from fedmi.data.tabular import DEFAULT_DATASET, DEFAULT_LABEL, load_tabular
from fedmi.fl.engine import EngineConfig
from fedmi.fl.trainer import FederatedMLPLearning
from fedmi.models.mlp import MLPModel  # noqa: F401  (reference symbol)
from fedmi.obs.console import JsonlWriter
from fedmi.parallel.comm import get_world
from fedmi.runtime.fault import parse_fault



def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data", default=DEFAULT_DATASET)
    ap.add_argument("--label", default=DEFAULT_LABEL)
    ap.add_argument("--rounds", type=int, default=300)
    ap.add_argument("--hidden", type=int, nargs="+", default=[50, 200])
    ap.add_argument("--lr", type=float, default=0.004)
    ap.add_argument("--step-size", type=int, default=30)
    ap.add_argument("--gamma", type=float, default=0.5)
    ap.add_argument("--local-steps", "--local-epochs", dest="local_steps", type=int, default=1,
                    help="local full-batch Adam steps per round (= local epochs: one step is one pass over the "
                         "shard, C:63-73)")
    ap.add_argument("--clients", type=int, default=0,
                    help="simulate K clients in THIS process (fedmi.fl.simulate.ClientGroup: K engines, FedAvg as an "
                         "in-process rank-order sum) instead of one client per process; 0 = one per process")
    ap.add_argument("--synthetic", action="store_true",
                    help="train on --synthetic-rows income-shaped rows per client (device Philox generator, 15 %% "
                         "label noise) instead of the CSV")
    ap.add_argument("--fedprox-mu", type=float, default=0.0)
    ap.add_argument("--participation", type=float, default=1.0,
                    help="fraction of clients sampled per round (both engines; 1.0 = all, the reference)")
    ap.add_argument("--patience", type=int, default=10)
    ap.add_argument("--tolerance", type=float, default=1e-4)
    ap.add_argument("--no-early-stop", action="store_true")
    ap.add_argument("--mode", choices=["compat", "correct"], default="compat")
    ap.add_argument("--partition", choices=["compat", "iid", "contiguous", "label_skew"], default=None)
    ap.add_argument("--alpha", type=float, default=0.5, help="Dirichlet alpha for label_skew")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--backend", default="auto", help="comm backend: rccl | nccl | gloo")
    ap.add_argument("--engine", default="auto", help="hip | torch")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="MFMA operand type of the fused HIP kernels (fp32 accumulate either way)")
    ap.add_argument("--rows-per-block", type=int, default=0, help="rows per workgroup: 16 | 32 | 0 = auto")
    ap.add_argument("--graph-rounds", type=int, default=16)
    ap.add_argument("--jsonl", default=None, help="append per-round metrics as JSON lines")
    ap.add_argument("--save", default=None, help="checkpoint directory written at the end (reference weight layout)")
    ap.add_argument("--resume", default=None, help="checkpoint directory to continue from (same clients/dims)")
    ap.add_argument("--fault-inject", default=None, metavar="RANK:ROUND[:raise|exit|hang]",
                    help="make one client fail at a round (tests the abort path)")
    ap.add_argument("--watchdog-s", type=float, default=300.0,
                    help="abort the job (non-zero exit on every rank) if a chunk of rounds stalls this long; 0 = off. "
                         "The xGMI data plane fails fast by itself (--peer-timeout-s); this is the host-side backstop")
    ap.add_argument("--peer-timeout-s", type=float, default=None,
                    help="seconds a device wait of the xGMI data plane waits for a peer before it reports the peer "
                         "as failed to every rank and the job aborts (default $FEDMI_PEER_TIMEOUT_S or 60)")
    ap.add_argument("--debug", action="store_true", help="synchronised phases + NaN/Inf checks every round")
    ap.add_argument("--profile", type=int, default=0, metavar="N",
                    help="time the first N rounds per phase with hipEvents (HIP engine)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--timing", action="store_true",
                    help="rank 0 prints main()'s wall time and BASELINE's end-to-end metric: shard rows x rounds "
                         "run / main() wall (CSV load, set-up and console included)")
    ap.add_argument("--wide", action="store_true",
                    help="BASELINE config 3: layer-by-layer wide-MLP client (e.g. --hidden 4096 4096 4096) on "
                         "device-generated synthetic shards of --synthetic-rows rows per client")
    ap.add_argument("--synthetic-rows", type=int, default=131072, help="rows per client for --wide")
    ap.add_argument("--micro-batch", type=int, default=131072,
                    help="rows per micro-batch for --wide (about 112 KiB of activation buffers per row at 4096 wide: 14 GiB of HBM)")
    ap.add_argument("--eval-every", type=int, default=0, help="--wide: local accuracy every N rounds")
    ap.add_argument("--wide-allreduce", default="fp32", choices=["fp32", "bf16"],
                    help="--wide: FedAvg bucket dtype on the wire (bf16: the round's delta, fp32 master weights "
                         "either way)")
    ap.add_argument("--wide-lr", type=float, default=None,
                    help="--wide: Adam learning rate (default fedmi.fl.wide.WIDE_LR = 1e-4: the reference's 0.004 "
                         "makes the 4096-wide model diverge, in torch as on the kernels, profiles/wide_learn_r3.log)")
    ap.add_argument("--wide-warmup", type=int, default=0, help="--wide: linear LR warm-up rounds")
    return ap.parse_args(argv)


def main_wide(a, comm):
    """--wide: federated wide-MLP rounds (fedmi.fl.wide.run_wide_fedavg)."""
    from fedmi.fl.wide import WIDE_LR, run_wide_fedavg
    dims = [14, *a.hidden, 2]
    res = run_wide_fedavg(comm, dims, a.synthetic_rows, a.rounds, micro_batch=a.micro_batch, dtype=a.dtype,
                          lr=a.wide_lr if a.wide_lr is not None else WIDE_LR, eval_every=a.eval_every,
                          seed=a.seed + 7, verbose=not a.quiet, allreduce_dtype=a.wide_allreduce,
                          warmup_rounds=a.wide_warmup)
    if comm.rank == 0 and comm.rccl_env:
        print(f"RCCL pinned: {comm.rccl_env}", flush=True)
    if comm.rank == 0:
        print(f"wide MLP {'-'.join(map(str, dims))}, {comm.size} client(s) x {a.synthetic_rows} rows: "
              f"{res['median_round_s'] * 1e3:.1f} ms/round, {res['tflops_per_client']:.1f} TFLOP/s per client, "
              f"{res['samples_per_s_per_client'] / 1e6:.2f} M samples/s/client", flush=True)
        if a.jsonl:
            w = JsonlWriter(a.jsonl)
            w.write(script="C-wide", dims=dims, clients=comm.size, **res)
            w.close()
    comm.close()
    return res


def _dataset(a, comm):
    """--synthetic: this client's shard of income-shaped rows, generated where it trains (on the
    GPU by the Philox kernel, rows [rank n, (rank + 1) n) of one stream; numpy on CPU), plus a
    held-out slice of the same distribution for --mode correct."""
    from types import SimpleNamespace
    n = int(a.synthetic_rows)
    if comm.device.type == "cuda":
        from fedmi.data.synthetic import device_shard
        X, y = device_shard(n, comm.rank, comm.device, seed=a.seed + 7)
        Xt, yt = device_shard(max(n // 4, 1), comm.size + comm.rank, comm.device, seed=a.seed + 7)
        Xt, yt = Xt.cpu().numpy(), yt.cpu().numpy().astype(np.int64)
    else:
        from fedmi.data.synthetic import make_income_like
        X, y = make_income_like(n, seed=a.seed * 1000 + comm.rank)
        Xt, yt = make_income_like(max(n // 4, 1), seed=a.seed * 1000 + 999)
    return SimpleNamespace(X_train=X, y_train=y, X_test=Xt, y_test=yt)


def main_clients(a, comm):
    """--clients K: K clients of one federation in this process (reference semantics client for
    client: own shard, local step, local evaluation, sample-weighted FedAvg, early stop on the
    mean of the clients' metrics), reference console output."""
    from fedmi.fl.simulate import ClientGroup
    from fedmi.obs.console import print_history
    if comm.Get_size() > 1:
        raise SystemExit("--clients simulates a federation in one process; launch it without torchrun / mpiexec")
    if a.save or a.resume or a.participation < 1.0:
        raise SystemExit("--clients does not combine with --save / --resume / --participation")
    ds = load_tabular(a.data, label=a.label, with_mean=True)
    cfg = EngineConfig(hidden=tuple(a.hidden), lr=a.lr, step_size=a.step_size, gamma=a.gamma,
                       local_steps=a.local_steps, prox_mu=a.fedprox_mu, early_stop=not a.no_early_stop,
                       patience=a.patience, tolerance=a.tolerance, max_rounds=a.rounds, seed=a.seed, dtype=a.dtype)
    backend = a.engine if a.engine != "auto" else ("hip" if comm.device.type == "cuda" else "torch")
    shard = a.partition or ("compat" if a.mode == "compat" else "iid")
    g = ClientGroup(ds.X_train, ds.y_train, a.clients, cfg, backend=backend, shard_mode=shard, seed=a.seed,
                    alpha=a.alpha, device=comm.device if backend == "hip" else None)
    t0 = time.perf_counter()
    g.run(a.rounds)
    wall = time.perf_counter() - t0
    h = g.history()
    if not a.quiet:
        print_history(h, a.patience)
    print(f"{a.clients} simulated clients ({backend}): {h['rounds_run']} rounds in {wall:.2f} s", flush=True)
    if a.jsonl:
        w = JsonlWriter(a.jsonl)
        w.history(h, clients=a.clients, script="C-clients", aggregation="in-process", wall_s=wall)
        w.close()
    comm.close()
    return h


def main(argv=None):
    t_main = time.perf_counter()
    a = parse_args(argv)
    if a.peer_timeout_s is not None:
        os.environ["FEDMI_PEER_TIMEOUT_S"] = str(a.peer_timeout_s)   # read by fedmi.parallel.peer
    if not 0.0 < a.participation <= 1.0:
        raise SystemExit("--participation must be in (0, 1]")
    if a.wide and a.participation < 1.0:
        raise SystemExit("--participation < 1 is not supported with --wide (every wide client trains every round)")
    # RCCL protocol pinned per workload: LL for the fused engine's small FedAvg images, Simple
    # for the wide MLP's large buckets (fedmi.parallel.comm.pin_rccl_env)
    comm = get_world(backend=a.backend, device=a.device, rccl_proto="Simple" if a.wide else "LL")
    t_comm = time.perf_counter()
    if a.wide:
        return main_wide(a, comm)
    rank, size = comm.Get_rank(), comm.Get_size()
    if a.clients:
        return main_clients(a, comm)

    # every rank derives the same split locally: no broadcast of the table (C:243-246)
    ds = _dataset(a, comm) if a.synthetic else load_tabular(a.data, label=a.label, with_mean=True)
    t_data = time.perf_counter()
    cfg = EngineConfig(hidden=tuple(a.hidden), lr=a.lr, step_size=a.step_size, gamma=a.gamma,
                       local_steps=a.local_steps, prox_mu=a.fedprox_mu, participation=a.participation, early_stop=not a.no_early_stop,
                       patience=a.patience, tolerance=a.tolerance, max_rounds=a.rounds,
                       rows_per_block=a.rows_per_block, graph_rounds=a.graph_rounds, seed=a.seed,
                       debug=a.debug, dtype=a.dtype)
    trainer = FederatedMLPLearning(ds.X_train, ds.y_train, rank, size, comm=comm, hidden_sizes=a.hidden,
                                   mode=a.mode, backend=a.engine, seed=a.seed, config=cfg,
                                   shard_mode=a.partition, alpha=a.alpha, presharded=a.synthetic,
                                   output_size=2 if a.synthetic else None,
                                   n_total=a.synthetic_rows * size if a.synthetic else None)
    t_setup = time.perf_counter()
    done = 0   # rounds restored from a checkpoint (not run by this process)
    if a.resume:
        done = resume(a.resume, trainer)
        if rank == 0:
            print(f"Resumed from {a.resume} after {done} rounds", flush=True)
    timings = None
    if a.profile and hasattr(trainer.engine, "profile"):
        timings = trainer.engine.profile(a.profile)
        if rank == 0:
            print("Phase timings (us/round, first %d rounds): " % a.profile
                  + ", ".join(f"{k}: {v:.2f}" for k, v in timings.items()), flush=True)
    t_train = time.perf_counter()
    global_metrics = trainer.train_and_evaluate(comm, rounds=a.rounds, termination_patience=a.patience,
                                                tolerance=a.tolerance, verbose=not a.quiet,
                                                fault=parse_fault(a.fault_inject), watchdog_s=a.watchdog_s)
    t_train = time.perf_counter() - t_train
    if a.mode == "correct":
        test = trainer.evaluate_global(ds.X_test, ds.y_test, comm)
        if rank == 0:
            print("Held-out test metrics of the aggregated model: "
                  + ", ".join(f"{k}: {v:.4f}" for k, v in test.items()), flush=True)
    if rank == 0 and a.jsonl:
        w = JsonlWriter(a.jsonl)
        # run-level observability: data plane, bytes all-reduced per round and
        # client, wall-clock throughput of the whole loop (host logging included)
        eng = trainer.engine
        h = trainer.history()
        rounds_run = max(int(h["rounds_run"]) - done, 1)   # this process's rounds (not the resumed ones)
        comm_floats = int(eng.params[0].numel()) if hasattr(eng, "params") else int(eng.P + eng.world * eng.tail_stride)
        w.history(h, clients=size, script="C", timings=timings,
                  aggregation=getattr(eng, "aggregation", "host"),
                  allreduce_bytes_per_round=4 * comm_floats if size > 1 else 0,
                  wall_s=t_train, samples_per_s_per_client=len(trainer.X_local) * rounds_run / max(t_train, 1e-9))
        w.close()
    if a.save:
        save_checkpoint(a.save, trainer)   # collective: every client writes its optimizer state
    if a.timing and rank == 0:
        # BASELINE.md "[C] samples/s/client (e2e)": shard rows / (wall of main() / rounds run) --
        # the rounds THIS process ran: after --resume the history also counts the restored ones
        rounds_run = max(int(trainer.history()["rounds_run"]) - done, 1)
        wall = time.perf_counter() - t_main
        print(f"main() wall {wall:.3f} s for {rounds_run} rounds ({t_train:.3f} s in train_and_evaluate): "
              f"e2e {len(trainer.X_local) * rounds_run / wall:,.0f} samples/s/client", flush=True)
        print(f"main() phases: communicator {t_comm - t_main:.3f} s, data {t_data - t_comm:.3f} s, "
              f"trainer set-up {t_setup - t_data:.3f} s, train_and_evaluate {t_train:.3f} s", flush=True)
    comm.close()
    return global_metrics


if __name__ == "__main__":
    main(sys.argv[1:])
