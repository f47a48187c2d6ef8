"""Several federated clients in ONE process (simulation mode).

The deployment model is one process per GPU, each GPU one client (``fedmi.parallel.comm``).
Some studies need more clients than processes -- the rounds-to-target distributions at
k = 2/4/8 on a one-GPU box, k > 8 clients on one node, quick CPU oracles -- so this module
runs k clients' round engines side by side in one process and replaces the cross-process
all-reduce with an in-process sum of their FedAvg buffers in rank order (the same left fold
the one-shot xGMI kernel uses, so the result equals a real k-rank run's arithmetic).

Semantics are the reference's, client for client: every client owns its shard
(``_split_data``, FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:48-61), trains
(C:145), evaluates its post-step local model (C:148), and all clients adopt the
sample-weighted average (C:101-120); the global metrics / early-stop rule see every
client's tail (C:165-192).

* ``backend='hip'``: k :class:`~fedmi.fl.engine.HipRoundEngine` on one device stream, classic
  rounds (train + Adam + eval kernels per client), the k FedAvg buffers summed on the device.
* ``backend='torch'``: k :class:`~fedmi.fl.engine.TorchRoundEngine` (CPU oracle).
"""
from __future__ import annotations

import copy
from typing import List, Optional

import numpy as np
import torch

from ..data.sharding import shard_indices
from ..models.mlp import init_flat
from .engine import EngineConfig, HipRoundEngine, TorchRoundEngine


class SimRank:
    """Stand-in communicator of one simulated client: rank / size / device only.  The
    collective is performed by :class:`ClientGroup`."""

    peer_allreduce = False
    native = None

    def __init__(self, size: int, rank: int, device):
        self.size, self.rank, self.device = int(size), int(rank), torch.device(device)

    def Barrier(self) -> None:  # the group's clients run in program order
        pass


class ClientGroup:
    """k clients of one federation in this process."""

    def __init__(self, X, y, k: int, cfg: EngineConfig, backend: str = "hip", shard_mode: str = "compat",
                 seed: int = 0, alpha: float = 0.5, device=None, n_classes: Optional[int] = None):
        X = np.asarray(X)
        y = np.asarray(y)
        self.k = int(k)
        self.backend = backend
        n_classes = int(n_classes if n_classes is not None else len(np.unique(y)))
        idx = [shard_indices(len(X), r, self.k, mode=shard_mode, seed=seed, labels=y, alpha=alpha)
               for r in range(self.k)]
        n_total = int(sum(len(i) for i in idx))
        dims = [int(X.shape[1]), *[int(h) for h in cfg.hidden], n_classes]
        if backend == "hip":
            self.device = torch.device(device if device is not None else "cuda")
        else:
            self.device = torch.device("cpu")
        self.clients: List = []
        for r in range(self.k):
            c = copy.deepcopy(cfg)
            if backend == "hip":
                c.lagged_eval = False    # classic rounds: each client evaluates itself
                c.graph_rounds = 0
            comm = SimRank(self.k, r, self.device)
            # FederatedMLPLearning's seeding: one init stream per (seed, rank)
            flat0 = init_flat(dims, seed * 1000003 + r)
            if backend == "hip":
                e = HipRoundEngine(X[idx[r]], y[idx[r]], n_classes, c, comm, flat0, n_total=n_total,
                                   device=self.device, client_sizes=[len(i) for i in idx])
            elif backend == "torch":
                e = TorchRoundEngine(X[idx[r]], y[idx[r]], n_classes, c, comm, flat0, n_total=n_total)
            else:
                raise ValueError(f"unknown backend {backend!r}")
            self.clients.append(e)
        if backend == "hip":
            self.stream = torch.cuda.Stream(device=self.device)
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            for e in self.clients:
                e.stream = self.stream   # one stream: every client's kernels and the sums in order
        self.rounds = 0

    # ---- rounds ----
    def _round_hip(self, r: int) -> None:
        s = self.stream.cuda_stream
        for e in self.clients:
            e.engine.run_local(r, s)      # train + Adam + eval into its own FedAvg buffer
        with torch.cuda.stream(self.stream):
            bufs = [e.params[(r + 1) & 1] for e in self.clients]
            tot = getattr(self, "_tot", None)
            if tot is None or tot.shape != bufs[0].shape:
                tot = self._tot = torch.empty_like(bufs[0])   # one accumulation buffer for all rounds
            tot.copy_(bufs[0])
            for b in bufs[1:]:
                tot += b                  # rank order
            for b in bufs:
                b.copy_(tot)
        for e in self.clients:
            e.rounds_issued = r + 1

    def _round_torch(self) -> None:
        for e in self.clients:
            e.step_train()
            e.step_eval()
        bufs = [e.fedavg_contribution() for e in self.clients]
        tot = bufs[0].clone()
        for b in bufs[1:]:
            tot += b
        for e in self.clients:
            e.fedavg_apply(tot.clone())

    @property
    def stopped(self) -> bool:
        return bool(self.clients[0].stopped)

    def run(self, n_rounds: int, check_every: int = 32) -> int:
        lead = self.clients[0]
        before = self.rounds
        left = min(n_rounds, lead.cfg.max_rounds - self.rounds)
        while left > 0 and not self.stopped:
            n = min(left, check_every)
            for _ in range(n):
                if self.backend == "hip":
                    self._round_hip(self.rounds)
                else:
                    if self.stopped:
                        break
                    self._round_torch()
                self.rounds += 1
            left -= n
            if self.backend == "hip":
                st = lead._read_state(self.rounds & 1)
                if st["stopped"]:
                    lead._stopped_seen = True
        self.sync_history()
        return self.rounds - before

    def sync_history(self) -> None:
        if self.backend == "hip":
            for e in self.clients:
                e.sync_history()

    def history(self) -> dict:
        return self.clients[0].history()

    def global_flat(self) -> np.ndarray:
        return self.clients[0].global_flat()


def rounds_to_target(X, y, k: int, cfg: EngineConfig, backend: str = "hip", seed: int = 0,
                     targets=(0.80, 0.83), shard_mode: str = "compat") -> dict:
    """Reference-compat convergence of k clients: first round reaching each global-accuracy
    target, the early-stop round and the final accuracy."""
    g = ClientGroup(X, y, k, cfg, backend=backend, shard_mode=shard_mode, seed=seed)
    g.run(cfg.max_rounds)
    h = g.history()
    acc = h["global"][:, 0]
    out = {}
    for t in targets:
        hit = np.flatnonzero(acc >= t)
        out[f"{t:.2f}"] = int(hit[0]) + 1 if len(hit) else None
    out["early_stop_round"] = int(h["stop_round"]) if h["stop_round"] >= 0 else None
    out["final_acc"] = float(acc[-1]) if len(acc) else None
    out["rounds_run"] = int(h["rounds_run"])
    return out
