"""Federated hyperparameter sweep over the round engine with concurrent trials per GPU
(BASELINE config 5: "8 clients x {lr, local_epochs, hidden_dim} grid, concurrent trials
packed per GPU").

The reference's sweep ([H], ``hyperparameters_tuning.py:68-132``) is sklearn-based and
strictly sequential: each of its 90 trials is fitted, averaged and scored before the next
starts (SURVEY §2.5 "Trial parallelism: no").  Here a *trial* is a full multi-round FedAvg
run of the [C] workload (``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:122-207``)
with its own hidden sizes, learning rate and local steps per round, and a
:class:`FedTrialGroup` runs K trials concurrently on every GPU:

* each trial is a fused :class:`~fedmi.fl.engine.HipRoundEngine`; trials of the same shape
  (layer sizes, dtype) form a native ``TrialBatch`` that runs every kernel of a round ONCE
  for all of them, with a trial grid dimension (K x 250 workgroups instead of K launches of
  250 on a 256-CU chip; ``fl_engine.cpp``), different shapes run their batches on their own
  HIP streams, and a whole group round (all batches, fork/join, shared all-reduce) is one
  captured HIP graph;
* all trials' FedAvg buffers are slices of ONE device allocation, so a round of all K
  trials costs one all-reduce (the per-trial weights, metric tails and early-stop inputs
  ride together), instead of K latency-bound collectives;
* each trial keeps its own device-side early-stop state; a stopped trial's rounds are exact
  no-ops inside the shared collective.

On CPU (gloo plumbing config) trials fall back to :class:`~fedmi.fl.engine.TorchRoundEngine`
run one after another with their own all-reduces.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..fl.engine import EngineConfig, HipRoundEngine, TorchRoundEngine, comm_len
from ..fl.metrics import METRIC_NAMES
from ..models.mlp import init_flat

DEFAULT_HIDDEN: Tuple[Tuple[int, ...], ...] = ((50, 200), (100, 50), (50, 100))  # fit the fused engine in fp32 and bf16
DEFAULT_LRS: Tuple[float, ...] = (0.002, 0.004, 0.01)
DEFAULT_LOCAL_STEPS: Tuple[int, ...] = (1, 2)


@dataclass
class FedTrial:
    hidden: Tuple[int, ...]
    lr: float
    local_steps: int
    history: dict = field(default_factory=dict, repr=False)

    @property
    def final(self) -> Dict[str, float]:
        g = self.history.get("global")
        if g is None or len(g) == 0:
            return {k: float("nan") for k in METRIC_NAMES}
        return {k: float(g[-1][i]) for i, k in enumerate(METRIC_NAMES)}

    @property
    def rounds_run(self) -> int:
        return int(self.history.get("rounds_run", 0))


def grid(hidden: Sequence[Sequence[int]] = DEFAULT_HIDDEN, lrs: Sequence[float] = DEFAULT_LRS,
         local_steps: Sequence[int] = DEFAULT_LOCAL_STEPS) -> List[FedTrial]:
    return [FedTrial(tuple(int(x) for x in h), float(lr), int(ls))
            for h, lr, ls in itertools.product(hidden, lrs, local_steps)]


class FedTrialGroup:
    """K federated trials on this client's shard, advanced in lock-step rounds.

    HIP: a round of the whole group -- every trial's kernels forked onto its own stream, joined,
    then (several clients) one all-reduce over all trials' FedAvg buffers -- is captured ONCE
    into a HIP graph of ``group_graph_rounds`` rounds and replayed, so a group round costs one
    graph launch for all K trials instead of K x (2-3) kernel launches + stream fork/join from
    Python.  One client: the trials are ordinary fused engines (evaluation inside the next
    round's train kernel, no all-reduce); several: classic rounds sharing one collective."""

    def __init__(self, X, y, n_classes: int, trials: Sequence[FedTrial], comm, base: EngineConfig,
                 n_total: Optional[int] = None, backend: str = "auto", seed: int = 0, group_graph_rounds: int = 16,
                 batched: bool = True):
        self.trials = list(trials)
        self.comm = comm
        self.world = comm.size if comm is not None else 1
        rank = comm.rank if comm is not None else 0
        if backend == "auto":
            backend = "hip" if torch.cuda.is_available() and (comm is None or comm.device.type == "cuda") else "torch"
        self.backend = backend
        F = int(X.shape[1])
        self.engines = []
        self.buffers = None
        self.graph = None
        self.graph_rounds = int(group_graph_rounds)
        cfgs = [replace(base, hidden=t.hidden, lr=t.lr, local_steps=t.local_steps) for t in self.trials]
        flats = [init_flat([F, *t.hidden, n_classes], seed * 1000003 + rank) for t in self.trials]
        if backend == "hip":
            dev = comm.device if comm is not None else torch.device("cuda", torch.cuda.current_device())
            if self.world == 1:
                # no collective: every trial is a plain fused engine
                for cfg, flat in zip(cfgs, flats):
                    self.engines.append(HipRoundEngine(X, y, n_classes, cfg, None, flat, device=dev))
            else:
                lens = [comm_len([F, *t.hidden, n_classes], self.world) for t in self.trials]
                offs = np.concatenate([[0], np.cumsum([(n + 63) & ~63 for n in lens])]).astype(np.int64)
                self.buffers = [torch.zeros(int(offs[-1]), dtype=torch.float32, device=dev) for _ in range(2)]
                for i, (cfg, flat) in enumerate(zip(cfgs, flats)):
                    views = (self.buffers[0][offs[i]:offs[i] + lens[i]], self.buffers[1][offs[i]:offs[i] + lens[i]])
                    self.engines.append(HipRoundEngine(X, y, n_classes, cfg, comm, flat, n_total=n_total, device=dev,
                                                       comm_buffers=views))
            self.stream = torch.cuda.Stream(device=dev)
            self.stream.wait_stream(torch.cuda.current_stream(dev))
            self._native = comm.rccl() if (comm is not None and self.world > 1 and hasattr(comm, "rccl")) else None
            # trial batches: same-shape engines, local steps descending (TrialBatch's order)
            self.batches = []
            if batched:
                from ..ops import native
                groups: Dict[tuple, List[int]] = {}
                for i, t in enumerate(self.trials):
                    groups.setdefault((tuple(t.hidden), self.engines[i].cfg.dtype), []).append(i)
                for idx in groups.values():
                    idx = sorted(idx, key=lambda i: -self.engines[i].cfg.local_steps)
                    tb = native().TrialBatch([self.engines[i].engine for i in idx])
                    self.batches.append((tb, idx, torch.cuda.Stream(device=dev)))
        elif backend == "torch":
            for cfg, flat in zip(cfgs, flats):
                self.engines.append(TorchRoundEngine(X, y, n_classes, cfg, comm, flat, n_total=n_total))
        else:
            raise ValueError(f"unknown backend {backend!r}")
        self.rounds_issued = 0

    # ---- HIP rounds ----
    def _issue_group_round(self, r: int) -> None:
        """Round r of every trial on the group stream (fork/join), plus the shared all-reduce."""
        if self.batches:
            for tb, _, st in self.batches:
                st.wait_stream(self.stream)
                if self.world == 1:
                    tb.run(r, 1, st.cuda_stream, close=False)   # fused evaluation rounds
                else:
                    tb.run_local(r, st.cuda_stream)              # classic rounds, no collective
            for _, _, st in self.batches:
                self.stream.wait_stream(st)
        else:
            for e in self.engines:
                e.stream.wait_stream(self.stream)
                if self.world == 1:
                    e.engine.run(r, 1, e._stream(), None, close=False)   # fused evaluation round
                else:
                    e.engine.run_local(r, e._stream())                   # classic round, no collective
            for e in self.engines:
                self.stream.wait_stream(e.stream)
        if self.world > 1:
            buf = self.buffers[(r + 1) & 1]
            with torch.cuda.stream(self.stream):
                if self._native is not None:
                    self._native.allreduce_f32(buf.data_ptr(), buf.numel(), self.stream.cuda_stream)
                else:
                    self.comm.allreduce_(buf)

    def _capturable(self) -> bool:
        return self.graph_rounds >= 2 and (self.world == 1 or self._native is not None)

    def _steady(self) -> bool:
        return not any(e.engine.needs_eager_round() for e in self.engines)

    def _sync_histories(self) -> None:
        """Fold the pending metrics of every trial (one batched finalize per batch) and read
        the histories."""
        if self.batches:
            r = self.rounds_issued_dev
            for tb, _, st in self.batches:
                st.wait_stream(self.stream)
                tb.finalize(r, st.cuda_stream)
                self.stream.wait_stream(st)
            self.stream.synchronize()
            for e in self.engines:
                e.read_history()
        else:
            for e in self.engines:
                e.stream.wait_stream(self.stream)
                e.sync_history()

    def _issue_rounds_unjoined(self, r0: int, n: int) -> None:
        """One client (no shared all-reduce): rounds of different trial batches do not depend on
        each other, so each batch runs its ``n`` rounds back to back on its own stream and the
        streams join once at the end -- no per-round join that holds every batch to the slowest
        one.  Every batch issues exactly the launches of ``n`` group rounds, in the same order."""
        for tb, _, st in self.batches:
            st.wait_stream(self.stream)
            for r in range(r0, r0 + n):
                tb.run(r, 1, st.cuda_stream, close=False)   # fused evaluation rounds
        for _, _, st in self.batches:
            self.stream.wait_stream(st)

    def _capture(self) -> None:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            if self.world == 1 and self.batches:
                self._issue_rounds_unjoined(0, self.graph_rounds)
            else:
                for r in range(self.graph_rounds):   # parities 0, 1, ...: replayed from even rounds
                    self._issue_group_round(r)
        self.graph = g
        self._graph_flags = [e.engine.flags() for e in self.engines]

    def _run_hip(self, n_rounds: int) -> None:
        r, end = self.rounds_issued, self.rounds_issued + n_rounds
        G = self.graph_rounds
        while r < end:
            if self._capturable() and r % 2 == 0 and end - r >= G and self._steady():
                if self.graph is None:
                    self._capture()
                with torch.cuda.stream(self.stream):
                    self.graph.replay()
                # the replayed rounds' effect on each engine's round bookkeeping: the state the
                # captured rounds left (a finalize in between may have changed it)
                for e, f in zip(self.engines, self._graph_flags):
                    e.engine.set_flags(f)
                r += G
            else:
                self._issue_group_round(r)
                r += 1
            for e in self.engines:
                e.rounds_issued = r
        self.rounds_issued_dev = r
        self.stream.synchronize()
        self._sync_histories()

    def run(self, n_rounds: int) -> None:
        """Run ``n_rounds`` rounds of every trial (trials that stopped early idle)."""
        n_rounds = min(n_rounds, min(e.cfg.max_rounds for e in self.engines) - self.rounds_issued)
        if self.backend == "hip":
            self._run_hip(n_rounds)
        else:
            for e in self.engines:
                e.run(n_rounds)
        self.rounds_issued += n_rounds
        for t, e in zip(self.trials, self.engines):
            t.history = e.history()

    def best(self, key: str = "accuracy") -> FedTrial:
        i = METRIC_NAMES.index(key)
        return max(self.trials, key=lambda t: (t.history["global"][-1][i] if t.rounds_run else -1.0))


def run_fed_sweep(X_local, y_local, n_classes: int, comm, trials: Sequence[FedTrial], rounds: int = 50,
                  trials_per_gpu: int = 6, base: Optional[EngineConfig] = None, n_total: Optional[int] = None,
                  backend: str = "auto", seed: int = 0, on_group=None,
                  group_graph_rounds: int = 16) -> Tuple[FedTrial, List[FedTrial]]:
    """Run ``trials`` in groups of ``trials_per_gpu`` concurrent trials; returns (best, all)."""
    base = base or EngineConfig()
    base = replace(base, max_rounds=max(base.max_rounds, rounds))
    done: List[FedTrial] = []
    for g0 in range(0, len(trials), trials_per_gpu):
        group = FedTrialGroup(X_local, y_local, n_classes, trials[g0:g0 + trials_per_gpu], comm, base,
                              n_total=n_total, backend=backend, seed=seed, group_graph_rounds=group_graph_rounds)
        group.run(rounds)
        done.extend(group.trials)
        if on_group is not None:
            on_group(group)
    i = METRIC_NAMES.index("accuracy")
    best = max(done, key=lambda t: (t.history["global"][-1][i] if t.rounds_run else -1.0))
    return best, done
