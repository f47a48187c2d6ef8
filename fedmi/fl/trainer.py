"""``FederatedMLPLearning`` -- the reference's [C] client API on the fedmi round engine.

Mirrors ``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:28-207`` method by
method (``_split_data``, ``train_one_epoch``, ``evaluate_local``, ``get_weights``,
``set_weights``, ``federated_averaging``, ``train_and_evaluate``) and the
``MLPModel(14, [50, 200], 2)`` / Adam(0.004) / StepLR(30, 0.5) defaults (C:39-46).

Differences by design (each switchable):

* ``mode='compat'`` keeps the reference's semantics: per-rank overlapping shards
  (C:48-61; seeded instead of unseeded), local evaluation on the training
  shard (Q2), unweighted mean of per-rank metrics (Q3).  ``mode='correct'`` uses
  disjoint IID shards; held-out evaluation of the aggregated model is available through
  :meth:`evaluate_global`.
* ``train_and_evaluate`` does not bounce through the host every round: the engine runs
  the whole loop (device-side early stop, one all-reduce per round) and the reference
  console lines are printed from the metric history as chunks of <= 16 rounds complete
  (pinned-host mirror read while the next chunk runs, ``HipRoundEngine.run_streaming``).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch

from ..data.sharding import split_data
from ..models.mlp import dict_to_flat, flat_to_dict, init_flat
from ..obs.console import print_history
from .engine import EngineConfig, make_engine
from .metrics import METRIC_NAMES, metrics_from_confusion


class FederatedMLPLearning:
    def __init__(self, X, y, rank: int, size: int, comm=None, hidden_sizes: Sequence[int] = (50, 200),
                 output_size: Optional[int] = None, lr: float = 0.004, mode: str = "compat",
                 backend: str = "auto", seed: int = 0, config: Optional[EngineConfig] = None,
                 shard_mode: Optional[str] = None, alpha: float = 0.5, n_total: Optional[int] = None,
                 presharded: bool = False):
        self.rank = rank
        self.size = size
        self.comm = comm
        self.mode = mode
        self.seed = seed
        if shard_mode is None:
            shard_mode = "compat" if mode == "compat" else "iid"
        self.shard_mode = shard_mode
        self.alpha = alpha
        if presharded:
            self.X_local, self.y_local = X, y
        else:
            self.X_local, self.y_local = self._split_data(X, y, rank, size)
        self.input_size = int(self.X_local.shape[1])
        self.hidden_sizes = list(hidden_sizes)
        self.output_size = int(output_size if output_size is not None else len(np.unique(y)))
        cfg = config or EngineConfig()
        cfg.hidden = tuple(self.hidden_sizes)
        cfg.lr = lr if config is None else cfg.lr
        self.cfg = cfg
        dims = [self.input_size, *self.hidden_sizes, self.output_size]
        # reference: unseeded torch init per rank -> seeded per rank (different models
        # until the first FedAvg, like the reference)
        flat0 = init_flat(dims, seed * 1000003 + rank)
        self.engine = make_engine(self.X_local, self.y_local, self.output_size, cfg, comm, flat0,
                                  n_total=n_total, backend=backend)
        self.device = getattr(self.engine, "device", torch.device("cpu"))
        self.global_weights = None

    # ---- reference API ----
    def _split_data(self, X, y, rank, size, shuffle: bool = True):
        mode = self.shard_mode if shuffle else "contiguous"
        return split_data(np.asarray(X), np.asarray(y), rank, size, mode=mode, seed=self.seed, alpha=self.alpha)

    def train_one_epoch(self) -> None:
        """Local full-batch Adam step(s) + StepLR step (C:63-73)."""
        self.engine.step_train()

    def evaluate_local(self) -> Dict[str, float]:
        """Metrics of the post-step local model on the local shard (C:75-91)."""
        return metrics_from_confusion(self.engine.step_eval())

    def get_weights(self) -> Dict[str, np.ndarray]:
        return self.engine.get_weights()

    def set_weights(self, global_weights: Dict[str, np.ndarray]) -> None:
        self.engine.set_global_flat(dict_to_flat(global_weights, self.engine.dims))

    def federated_averaging(self, comm=None) -> None:
        """Sample-size-weighted FedAvg (C:101-120) as one in-place all-reduce."""
        self.engine.step_aggregate()
        self.global_weights = flat_to_dict(self.engine.global_flat(), self.engine.dims)

    def train_and_evaluate(self, comm=None, rounds: int = 5, termination_patience: int = 10,
                           tolerance: float = 1e-4, verbose: bool = True, chunk: int = 64,
                           fault=None, watchdog_s: float = 0.0, stream_chunk: int = 16):
        """Multi-round FedAvg with early stopping (C:122-207).  Returns the reference's
        ``global_metrics`` dict of per-round lists.

        ``fault`` (:class:`fedmi.runtime.FaultSpec`) injects a failure on one client at a
        given round; ``watchdog_s`` > 0 aborts the job when a chunk of rounds (kernels +
        all-reduces) stalls that long, e.g. because a peer died inside a collective."""
        from ..runtime.watchdog import Watchdog
        eng = self.engine
        comm = comm if comm is not None else self.comm
        if termination_patience != eng.cfg.patience or tolerance != eng.cfg.tolerance:
            eng.set_early_stop(termination_patience, tolerance)   # raises after the first round
        printed = eng.hist.rounds_run
        abort = (comm.Abort if comm is not None and hasattr(comm, "Abort") else (lambda: None))
        wd = Watchdog(watchdog_s, abort, rank=self.rank)
        # verbose: the console follows the rounds as they complete (every rank runs the same
        # chunking -- the collectives of the rounds must match -- and rank 0 prints):
        # run_streaming keeps one chunk of <= `stream_chunk` rounds in flight behind the printed ones
        stream = verbose and hasattr(eng, "run_streaming")

        announced = False   # the stop line is printed once (a chunk in flight past the stop re-reports it)

        def on_history(h):
            nonlocal printed, announced
            if self.rank == 0 and not announced:
                printed = print_history(h, termination_patience, start=printed)
                announced = h.get("stop_round", -1) >= 0 and printed == h["stop_round"]
        try:
            left = rounds - eng.rounds_issued
            while left > 0 and not eng.stopped:
                n = left if stream else min(chunk, left)
                if fault is not None:
                    # EVERY rank (the spec is on every command line) ends a run call at the fault
                    # round, so the ranks' chunking -- and with it the collectives of each round --
                    # stays identical up to the fault; only the faulting rank fails there
                    to_fault = fault.round - eng.rounds_issued
                    if to_fault <= 0 and fault.applies(self.rank):
                        fault.trigger(self.rank, eng.rounds_issued)
                    if to_fault > 0:
                        n = min(n, to_fault)
                if stream:
                    eng.run_streaming(n, chunk=stream_chunk, on_history=on_history, guard=wd.guard)
                else:
                    with wd.guard(f"rounds {eng.rounds_issued}..{eng.rounds_issued + n - 1}"):
                        eng.run(n)
                    if verbose:
                        on_history(eng.history())
                left -= n
        except Exception as e:  # reference C:203-205
            print(f"Rank {self.rank} encountered an error: {e}", flush=True)
            if comm is not None and hasattr(comm, "Abort") and getattr(comm, "size", 1) > 1:
                comm.Abort()
            raise
        finally:
            wd.close()
        gflat = eng.global_flat()
        self.global_weights = flat_to_dict(gflat, eng.dims)
        if comm is not None and getattr(comm, "size", 1) > 1:
            # every client must end the run holding the same global model and metric history
            # (C:119-120); a data-plane fault raises here instead of passing as a result
            from ..parallel.consistency import check_replicas
            eng.sync_history()
            self.replicas_consistent = check_replicas(comm, [gflat, np.asarray(eng.history()["global"])])
        else:
            self.replicas_consistent = True
        return eng.hist.global_metrics_dict()

    # ---- extras ----
    def evaluate_global(self, X_test, y_test, comm=None) -> Dict[str, float]:
        """Held-out evaluation of the aggregated model ('correct' mode), pooled over ranks."""
        cm = self.engine.confusion(X_test, y_test, flat=self.engine.global_flat())
        comm = comm or self.comm
        if comm is not None and comm.size > 1:
            t = torch.as_tensor(cm.astype(np.float64))
            import torch.distributed as dist
            dist.all_reduce(t)
            cm = t.numpy()
        return metrics_from_confusion(cm)

    def history(self) -> dict:
        return self.engine.history()

    @property
    def local_model_weights(self):
        return flat_to_dict(self.engine.local_flat(), self.engine.dims)


__all__ = ["FederatedMLPLearning", "METRIC_NAMES"]
