"""Round engines: one federated client's local train -> local eval -> FedAvg loop.

Two implementations with one interface and identical semantics:

* :class:`HipRoundEngine` -- the MI355X path.  Shard, flat parameters, Adam state, gradient
  slab, round state and metric history are device-resident; each round is three fused
  gfx950 kernels plus one RCCL all-reduce issued from C++ (``fedmi/ops/csrc``), optionally
  replayed as a captured HIP graph.  Early stopping is evaluated on the device.
* :class:`TorchRoundEngine` -- eager torch ops (``nn.Linear``, ``CrossEntropyLoss``,
  ``torch.optim.Adam`` + ``StepLR``), i.e. the reference's own numerics
  (``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:30-120``).  Used on CPU (the
  gloo plumbing config) and as the oracle the HIP kernels are tested against.

Round semantics (reference-compat): ``local_steps`` full-batch Adam steps
(reference: 1), StepLR stepped once per round, Adam moments never reset, local metrics of
the post-step model on the local *training* shard, global metrics = mean over clients of
local metrics (``metric_mode='mean'``, Q3) or pooled confusion (``'pooled'``, Q4),
weights averaged with weights n_i / N (C:110-116), early stop with patience/atol on the
4-metric vector (C:181-192).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, asdict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..models.mlp import (MLPModel, dense_to_image, flat_to_dict, image_layout, image_to_dense,
                          param_count)
from .early_stop import EarlyStopper
from .metrics import METRIC_NAMES, confusion_matrix, metrics_from_confusion, metric_vector


# bf16 shards of at most this many rows default to 16 rows per workgroup (EngineConfig.rows_per_block = 0):
# measured on MI355X (profiles/round_emulate_r4_shards.log), R = 16 wins at 1000 and 2000 rows,
# R = 32 at 4000 and 8000.
SMALL_SHARD_ROWS = 2000


@dataclass
class EngineConfig:
    hidden: Sequence[int] = (50, 200)
    lr: float = 0.004
    betas: Sequence[float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    step_size: int = 30
    gamma: float = 0.5
    local_steps: int = 1
    prox_mu: float = 0.0
    early_stop: bool = True
    patience: int = 10
    tolerance: float = 1e-4
    rtol: float = 1e-5
    max_rounds: int = 300
    metric_mode: str = "mean"       # 'mean' (C:169) | 'pooled' (S:130)
    rows_per_block: int = 0         # R rows per workgroup of the fused kernels (16 | 32 | 64 (bf16); 0 = auto:
                                    # 16 for bf16 shards of <= SMALL_SHARD_ROWS rows, else 32 if it fits LDS, else 16;
                                    # -1 = the largest that fits, 64 first (bf16))
    graph_rounds: int = 16          # rounds per captured HIP graph (0 = eager launches)
    seed: int = 0
    # partial participation (client sampling): each round max(1, round(participation * world))
    # clients, drawn by numpy's default Generator seeded with (seed, round) so every rank
    # draws the same set, train and are averaged (weights n_i / sum of the sampled n_i); the
    # others skip the local step and take the new global model.  The LR schedule follows the
    # round index for everyone, Adam's bias correction each client's own step count; global
    # metrics and loss are the sampled clients'.  Both engines (HIP: a per-round device table).
    participation: float = 1.0
    debug: bool = False             # eager, synchronised phases + non-finite checks every round
    dtype: str = "fp32"             # MFMA operand type of the fused kernels: 'fp32' | 'bf16'
    # one client: score round r's post-step model inside round r+1's train kernel (its forward
    # pass IS that evaluation, FedAvg of one client being the identity) instead of a separate
    # eval kernel; metrics, history and early stop are unchanged (fl_common.h FL_EVAL_FUSED)
    fused_eval: bool = True
    # world > 1 with the one-shot xGMI all-reduce: evaluate the post-step local model and
    # all-reduce in ONE kernel, the weights' all-reduce overlapping the evaluation
    # (fedmi/ops/csrc/peer_device.h); False = separate eval and all-reduce kernels
    eval_fedavg: bool = True
    # world > 1, bf16: score round r's post-step local model inside round r+1's train kernel --
    # no evaluation kernel in the round; the counts are exchanged inside round r+1's Adam
    # kernel (one-shot xGMI) or ride round r+1's all-reduce (RCCL; with early stopping a round
    # run past the stop is discarded bit-exactly, fl_common.h FLState::late); the
    # last round of every run() evaluates itself (fl_common.h FL_EVAL_LAGGED).  Metrics,
    # history, early-stop round and weights are identical to classic rounds.
    lagged_eval: bool = True
    # bf16 fused kernels: storage of the per-workgroup gradient partials reduced by the Adam
    # kernel -- 'fp16' (half the slab traffic; partial SUMS of the unscaled gradient, 1/n applied
    # after the fp32 reduction, saturating at +-65504), 'fp32', or 'auto' = fp16 when every
    # |feature| <= FP16_SLAB_MAX_ABS_X (standardised data: a partial over R <= 64 rows stays far
    # inside fp16's range), else fp32.  The fp32 kernels always use an fp32 slab.
    grad_slab: str = "auto"
    # bf16 kernels, several clients: run the TRAINING forward pass in plain bf16 (a_hi.W_hi) instead
    # of split-bf16 -- no round is scored from it there (lagged rounds score in registers, classic
    # rounds in the eval kernel, both split-bf16); None = auto (on for world > 1 / emulated
    # clients with register scoring), False = the split forward everywhere, True = on where it is
    # valid (never for one fused client, whose evaluation IS the training forward).  The engine's
    # layout()["plain_fwd"] reports what runs; bench records and checkpoints carry it.
    plain_fwd: Optional[bool] = None

    def to_dict(self) -> dict:
        d = asdict(self)
        d["hidden"] = list(self.hidden)
        d["betas"] = list(self.betas)
        return d


def _metric_mode_id(mode: str) -> int:
    if mode not in ("mean", "pooled"):
        raise ValueError(f"metric_mode must be 'mean' or 'pooled', got {mode!r}")
    return 0 if mode == "mean" else 1


# grad_slab='auto': the largest |feature| for which the bf16 kernels use fp16 gradient partials
FP16_SLAB_MAX_ABS_X = 64.0


def _dtype_id(dtype: str) -> int:
    if dtype not in ("fp32", "bf16"):
        raise ValueError(f"dtype must be 'fp32' or 'bf16', got {dtype!r}")
    return 0 if dtype == "fp32" else 1


class _History:
    def __init__(self, max_rounds: int, world: int):
        self.glob = np.zeros((max_rounds, 4))
        self.rank = np.zeros((max_rounds, world, 4))
        self.loss = np.zeros(max_rounds, dtype=np.float32)
        self.rounds_run = 0
        self.stop_round = -1       # round index at which training stopped early (-1: never)
        self.stop_trigger = -1     # round whose metrics triggered the stop

    def as_dict(self) -> dict:
        n = self.rounds_run
        return {
            "rounds_run": n,
            "stop_round": self.stop_round,
            "stop_trigger": self.stop_trigger,
            "global": self.glob[:n].copy(),
            "per_rank": self.rank[:n].copy(),
            "loss": self.loss[:n].copy(),
        }

    def global_metrics_dict(self) -> Dict[str, List[float]]:
        """Same structure as the reference's returned ``global_metrics`` (C:124)."""
        n = self.rounds_run
        return {k: [float(x) for x in self.glob[:n, i]] for i, k in enumerate(METRIC_NAMES)}


class RoundEngineBase:
    def __init__(self, X: np.ndarray, y: np.ndarray, n_classes: int, cfg: EngineConfig, comm,
                 init_flat: np.ndarray, n_total: Optional[int] = None):
        self.cfg = cfg
        self.comm = comm
        self.world = comm.size if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.n_local = int(len(X))
        if self.n_local == 0:
            raise ValueError("client shard is empty (reference SURVEY Q12 would deadlock)")
        self.dims = [int(X.shape[1]), *[int(h) for h in cfg.hidden], int(n_classes)]
        self.n_classes = int(n_classes)
        self.P = param_count(self.dims)
        if n_total is None:
            n_total = self._allreduce_scalar(float(self.n_local))
        self.n_total = int(n_total)
        self.agg_scale = float(self.n_local) / float(self.n_total)
        self.tail_stride = self.n_classes * self.n_classes + 1
        self.hist = _History(cfg.max_rounds, self.world)
        assert init_flat.shape == (self.P,)

    def participants(self, r: int) -> np.ndarray:
        """Ranks that train and are averaged in round r (all of them unless sampling): the same
        seeded draw on every rank, so no broadcast is needed."""
        frac = float(self.cfg.participation)
        if frac >= 1.0 or self.world == 1:
            return np.arange(self.world)
        k = max(1, int(round(frac * self.world)))
        rng = np.random.default_rng([int(self.cfg.seed), int(r)])
        return np.sort(rng.choice(self.world, size=k, replace=False))

    def own_steps(self, rounds: int) -> int:
        """Adam steps this client took in rounds [0, rounds) (it only steps when sampled)."""
        if float(self.cfg.participation) >= 1.0 or self.world == 1:
            return rounds * int(self.cfg.local_steps)
        return sum(int(self.rank in self.participants(r)) for r in range(rounds)) * int(self.cfg.local_steps)

    def set_early_stop(self, patience: int, tolerance: float) -> None:
        """Early-stop parameters of ``train_and_evaluate(termination_patience, tolerance)``
        (C:122); only before the first round."""
        if getattr(self, "rounds_issued", 0):
            raise RuntimeError("early-stop parameters must be set before the first round")
        self.cfg.patience = int(patience)
        self.cfg.tolerance = float(tolerance)
        self._apply_early_stop()

    def _apply_early_stop(self) -> None:
        raise NotImplementedError

    def _allreduce_scalar(self, x: float) -> float:
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        import torch.distributed as dist
        dist.all_reduce(t)
        return float(t.item())

    # subclass API
    def run(self, n_rounds: int) -> int:
        raise NotImplementedError

    def global_flat(self) -> np.ndarray:
        raise NotImplementedError

    def local_flat(self) -> np.ndarray:
        raise NotImplementedError

    def get_weights(self) -> Dict[str, np.ndarray]:
        return flat_to_dict(self.local_flat(), self.dims)

    def history(self) -> dict:
        return self.hist.as_dict()

    # -- resume (round index, Adam m/v, StepLR counter, early-stop state) --
    def portable_state(self) -> dict:
        """Engine-independent resume state (dense reference layout, numpy only).  A state
        written by one backend loads into the other."""
        raise NotImplementedError

    def load_portable_state(self, st: dict) -> None:
        raise NotImplementedError

    def _load_history(self, h: dict) -> None:
        n = int(h.get("rounds_run", 0))
        self.hist.rounds_run = n
        if n:
            self.hist.glob[:n] = np.asarray(h["global"], dtype=np.float64).reshape(n, 4)
            self.hist.rank[:n] = np.asarray(h["per_rank"], dtype=np.float64).reshape(n, self.world, 4)
            self.hist.loss[:n] = np.asarray(h["loss"], dtype=np.float32).reshape(n)
        self.hist.stop_round = int(h.get("stop_round", -1))
        self.hist.stop_trigger = int(h.get("stop_trigger", -1))


# ---------------------------------------------------------------------------------------
# Torch (CPU / oracle) engine
# ---------------------------------------------------------------------------------------
class TorchRoundEngine(RoundEngineBase):
    def __init__(self, X, y, n_classes, cfg: EngineConfig, comm, init_flat, n_total=None,
                 device="cpu", X_dtype=torch.float32):
        super().__init__(X, y, n_classes, cfg, comm, init_flat, n_total)
        self.device = torch.device(device)
        self.X = torch.as_tensor(np.asarray(X), dtype=X_dtype, device=self.device)
        self.y = torch.as_tensor(np.asarray(y), dtype=torch.long, device=self.device)
        self.model = MLPModel(self.dims[0], self.dims[1:-1], self.dims[-1], device=self.device)
        with torch.no_grad():
            self.model.flat.copy_(torch.as_tensor(init_flat))
        self.criterion = torch.nn.CrossEntropyLoss()
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=cfg.lr, betas=tuple(cfg.betas),
                                          eps=cfg.eps, weight_decay=cfg.weight_decay)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=cfg.step_size,
                                                         gamma=cfg.gamma)
        self.stopper = EarlyStopper(cfg.patience, cfg.tolerance, cfg.rtol, enabled=cfg.early_stop)
        self.global_params = self.model.flat.detach().clone()
        self.rounds_issued = 0

    def train_one_epoch(self) -> float:
        """``local_steps`` full-batch Adam steps + one StepLR step (reference C:63-73)."""
        self.model.train()
        anchor = self.model.flat.detach().clone() if self.cfg.prox_mu else None
        loss_v = 0.0
        for _ in range(self.cfg.local_steps):
            self.optimizer.zero_grad()
            out = self.model(self.X)
            loss = self.criterion(out, self.y)
            loss.backward()
            if anchor is not None:
                with torch.no_grad():
                    for (name, shape, off), p in zip(self.model.layout, self.model.parameters()):
                        n = int(np.prod(shape))
                        p.grad.add_(self.cfg.prox_mu * (p.detach() - anchor[off:off + n].view(shape)))
            self.optimizer.step()
            loss_v = float(loss.detach())
        self._scheduler_step()
        return loss_v

    def _scheduler_step(self) -> None:
        """StepLR follows the global round index (C:73 steps it once per round) for every
        client, sampled or not; only a sampled client's Adam takes a step."""
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)  # "scheduler.step() before optimizer.step()"
            self.scheduler.step()

    def confusion(self, X=None, y=None, flat=None) -> np.ndarray:
        Xt = self.X if X is None else torch.as_tensor(np.asarray(X), dtype=torch.float32, device=self.device)
        yt = self.y if y is None else torch.as_tensor(np.asarray(y), dtype=torch.long, device=self.device)
        model = self.model
        if flat is not None:
            model = MLPModel(self.dims[0], self.dims[1:-1], self.dims[-1], device=self.device)
            with torch.no_grad():
                model.flat.copy_(torch.as_tensor(flat))
        model.eval()
        with torch.no_grad():
            _, pred = torch.max(model(Xt), 1)
        return confusion_matrix(yt.cpu().numpy(), pred.cpu().numpy(), self.n_classes)

    def _apply_early_stop(self) -> None:
        cfg = self.cfg
        self.stopper = EarlyStopper(cfg.patience, cfg.tolerance, cfg.rtol, enabled=cfg.early_stop)

    # -- step-by-step API (reference train_one_epoch / evaluate_local / federated_averaging)
    def step_train(self) -> None:
        r = self.rounds_issued
        self._active = self.rank in self.participants(r)
        if self._active:
            self._loss = self.train_one_epoch()
        else:
            self._loss = 0.0
            self._scheduler_step()

    def step_eval(self) -> np.ndarray:
        self._cm = self.confusion()
        return self._cm

    def fedavg_contribution(self) -> torch.Tensor:
        """This client's operand of the round's SUM all-reduce:
        [w * n_i/N | per-rank (confusion, loss) tails] (+ n_i when sampling clients)."""
        sampling = float(self.cfg.participation) < 1.0 and self.world > 1
        buf = torch.zeros(self.P + self.world * self.tail_stride + int(sampling), dtype=torch.float32)
        if not sampling:
            buf[:self.P] = self.model.flat.detach().cpu() * self.agg_scale
        elif getattr(self, "_active", True):
            # weights n_i * w_i and, in the last slot, n_i: divided by the sampled total after the sum
            buf[:self.P] = self.model.flat.detach().cpu() * float(self.n_local)
            buf[-1] = float(self.n_local)
        t0 = self.P + self.rank * self.tail_stride
        buf[t0:t0 + self.n_classes ** 2] = torch.as_tensor(self._cm.reshape(-1), dtype=torch.float32)
        buf[t0 + self.n_classes ** 2] = self._loss
        return buf

    def step_aggregate(self) -> None:
        # one SUM all-reduce of [w * n_i/N | per-rank (confusion, loss) tails]
        buf = self.fedavg_contribution()
        if self.comm is not None:
            self.comm.allreduce_(buf)
        self.fedavg_apply(buf)

    def fedavg_apply(self, buf: torch.Tensor) -> None:
        """Adopt the all-reduced buffer: new global weights, metrics, early-stop rule."""
        r = self.rounds_issued
        sampling = float(self.cfg.participation) < 1.0 and self.world > 1
        if sampling:
            buf[:self.P] /= buf[-1]
            buf = buf[:-1]
        with torch.no_grad():
            self.model.flat.copy_(buf[:self.P].to(self.device))
        self.global_params = self.model.flat.detach().clone()
        self._finalize(r, buf[self.P:].numpy())
        self.rounds_issued += 1

    def run(self, n_rounds: int) -> int:
        ran = 0
        for _ in range(n_rounds):
            if self.stopper.stopped or self.rounds_issued >= self.cfg.max_rounds:
                break
            self.step_train()
            self.step_eval()
            self.step_aggregate()
            ran += 1
        return ran

    def sync_history(self) -> None:
        pass

    def run_streaming(self, n_rounds: int, chunk: int = 16, on_history=None, guard=None) -> int:
        """:meth:`run` round by round, ``on_history`` after every round (host-driven rounds: each
        round's metrics are on the host as soon as it ends)."""
        import contextlib
        ran = 0
        for _ in range(int(n_rounds)):
            if self.stopper.stopped or self.rounds_issued >= self.cfg.max_rounds:
                break
            with (guard(f"round {self.rounds_issued}") if guard else contextlib.nullcontext()):
                ran += self.run(1)
            if on_history is not None:
                on_history(self.history())
        return ran

    @property
    def stopped(self) -> bool:
        return self.stopper.stopped

    def _finalize(self, r: int, tail: np.ndarray) -> None:
        if self.cfg.debug:
            _check_finite(r, "aggregated weights", self.model.flat.detach())
            _check_finite(r, "loss/confusion tail", torch.as_tensor(tail))
        tails = tail.reshape(self.world, self.tail_stride)
        C = self.n_classes
        per = [metrics_from_confusion(t[:C * C].reshape(C, C)) for t in tails]
        # global metrics / loss: the round's sampled clients (every client without sampling);
        # per-client metrics are recorded for all (an unsampled client scores the global model)
        part = self.participants(r)
        if self.cfg.metric_mode == "mean":
            g = metric_vector({k: float(np.mean([per[i][k] for i in part])) for k in METRIC_NAMES})
        else:
            g = metric_vector(metrics_from_confusion(tails[part, :C * C].sum(0).reshape(C, C)))
        self.hist.glob[r] = g
        self.hist.rank[r] = np.stack([metric_vector(m) for m in per])
        self.hist.loss[r] = float(tails[part, C * C].astype(np.float64).sum() / len(part))
        self.hist.rounds_run = r + 1
        if self.stopper.update(g):
            self.hist.stop_trigger = r
            self.hist.stop_round = r + 1

    def global_flat(self) -> np.ndarray:
        return self.global_params.cpu().numpy().copy()

    def local_flat(self) -> np.ndarray:
        return self.model.flat.detach().cpu().numpy().copy()

    def set_global_flat(self, flat: np.ndarray) -> None:
        with torch.no_grad():
            self.model.flat.copy_(torch.as_tensor(flat))
        self.global_params = self.model.flat.detach().clone()

    def state_dict(self) -> dict:
        return {"params": self.global_flat(), "optimizer": self.optimizer.state_dict(),
                "scheduler": self.scheduler.state_dict(), "stopper": self.stopper.state_dict(),
                "rounds": self.rounds_issued, "history": self.hist.as_dict()}

    def portable_state(self) -> dict:
        params = list(self.model.parameters())
        m = [self.optimizer.state.get(p, {}).get("exp_avg") for p in params]
        v = [self.optimizer.state.get(p, {}).get("exp_avg_sq") for p in params]
        cat = (lambda ts: np.zeros(self.P, np.float32) if ts[0] is None else
               torch.cat([t.detach().reshape(-1).cpu() for t in ts]).numpy().astype(np.float32))
        sp = self.stopper
        st0 = self.optimizer.state.get(params[0], {}).get("step")
        return {
            "rounds": int(self.rounds_issued), "global": self.global_flat(), "local": self.local_flat(),
            "exp_avg": cat(m), "exp_avg_sq": cat(v), "opt_steps": int(st0) if st0 is not None else 0,
            "es": {"count": int(sp.count), "has_prev": sp.prev is not None,
                   "prev": [0.0] * 4 if sp.prev is None else [float(x) for x in sp.prev],
                   "stopped": bool(sp.stopped), "stop_round": int(self.hist.stop_round)},
            "history": self.hist.as_dict(),
        }

    def load_portable_state(self, st: dict) -> None:
        r = int(st["rounds"])
        cfg = self.cfg
        with torch.no_grad():
            self.model.flat.copy_(torch.as_tensor(np.asarray(st["global"], np.float32)))
        self.global_params = self.model.flat.detach().clone()
        steps = int(st.get("opt_steps", self.own_steps(r)))   # this client's own Adam steps
        if steps:
            off = 0
            for p in self.model.parameters():
                n = p.numel()
                self.optimizer.state[p] = {
                    "step": torch.tensor(float(steps)),
                    "exp_avg": torch.as_tensor(np.asarray(st["exp_avg"][off:off + n], np.float32)).view_as(p).clone(),
                    "exp_avg_sq": torch.as_tensor(np.asarray(st["exp_avg_sq"][off:off + n], np.float32)).view_as(p).clone(),
                }
                off += n
        lr = cfg.lr * cfg.gamma ** (r // cfg.step_size)
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        self.scheduler.last_epoch = r
        self.scheduler._step_count = r + 1
        self.scheduler._last_lr = [lr]
        es = st["es"]
        self.stopper.count = int(es["count"])
        self.stopper.prev = np.asarray(es["prev"], np.float64) if es["has_prev"] else None
        self.stopper.stopped = bool(es["stopped"])
        self.rounds_issued = r
        self._load_history(st["history"])


# ---------------------------------------------------------------------------------------
# HIP engine
# ---------------------------------------------------------------------------------------
_STATE_DTYPE = np.dtype([("next_round", "<i4"), ("finalized", "<i4"), ("stopped", "<i4"), ("live", "<i4"),
                         ("cur_round", "<i4"), ("count", "<i4"), ("has_prev", "<i4"), ("stop_round", "<i4"),
                         ("calls", "<u4"), ("late", "<i4"), ("prev", "<f8", (4,))])


class HipRoundEngine(RoundEngineBase):
    """Device-resident client.  ``X``/``y`` may be numpy arrays (uploaded once) or CUDA
    tensors already on the device (e.g. from the synthetic generator)."""

    def __init__(self, X, y, n_classes, cfg: EngineConfig, comm, init_flat, n_total=None, device=None,
                 comm_buffers=None, emulate_clients: bool = False, client_sizes=None, stream=None):
        """``stream``: the torch stream the engine issues on (default: a new one).  Engines created one
        after another in a process (bench.py's timed runs) should share one: with ranks sharing a
        GPU, a second engine on a fresh stream ran its Adam-exchange rounds 2.3x slower
        (108 vs 46 us per round, profiles/bench_r4_n2_share_stream.log).
        ``comm_buffers``: optional pair of float32 device views of length
        :meth:`comm_len` to use as the double-buffered FedAvg buffers (trial packing shares one
        all-reduce between engines by handing each a slice of one allocation).
        ``client_sizes``: every client's shard size (client sampling weighs the sampled clients
        by n_i / their sum); gathered over ``comm`` when needed and not given."""
        from ..ops import native
        self.m = native()
        if device is None:
            device = comm.device if comm is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if isinstance(X, torch.Tensor):
            Xn_len = X.shape[0]
            Xshape1 = X.shape[1]
        else:
            Xn_len, Xshape1 = X.shape
        super().__init__(_ShapeOnly(Xn_len, Xshape1), y, n_classes, cfg, comm, init_flat, n_total)
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.X = (X if isinstance(X, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(X, np.float32))).to(**f32).contiguous()
        self.y = (y if isinstance(y, torch.Tensor) else torch.as_tensor(np.asarray(y))).to(dtype=torch.int32, device=dev).contiguous()
        # rows per workgroup: 0 = auto (32 when the model's LDS image fits, else 16); -1 = the
        # largest that fits, 64 first (bf16: half the workgroups and gradient-slab rows -- what
        # packed trial batches want, whose throughput is workgroup-slots x workgroup latency)
        rpb = int(cfg.rows_per_block)
        # (auto: small shards -- the reference's 8000 // k rows at k >= 4 -- run twice the
        # workgroups at 16 rows each, lower per-workgroup latency; profiles/round_emulate_r4_shards.log)
        auto = [16, 32] if (Xn_len <= SMALL_SHARD_ROWS and cfg.dtype == "bf16") else [32, 16]
        R_try = auto if rpb == 0 else ([64, 32, 16] if cfg.dtype == "bf16" else [32, 16]) if rpb == -1 else [rpb]
        R = R_try[0]
        slab_stride = ((self.P + 1) + 3) & ~3
        # device parameter buffers use the padded image layout (fl_common.h)
        self.Pimg = image_layout(self.dims)[2]
        # lagged evaluation carries a second metric region after the tails (fl_common.h)
        # (emulate_clients: one process measures the multi-client round shape, tools/round_emulate.py)
        # (with early stopping the native engine runs lagged rounds with the Adam-fused exchange,
        # which folds each round's metrics in time, or over RCCL, folded one round late with the
        # round run past a stop discarded bit-exactly: FLEngine.late_fold)
        self._lag = ((self.world > 1 or emulate_clients) and cfg.dtype == "bf16"
                     and comm_buffers is None and bool(cfg.lagged_eval))
        comm_len = self.Pimg + self.world * self.tail_stride * (2 if self._lag else 1)
        if comm_buffers is None:
            self.params = [torch.zeros(comm_len, **f32), torch.zeros(comm_len, **f32)]
        else:
            self.params = list(comm_buffers)
            for t in self.params:
                if t.numel() != comm_len or t.dtype != torch.float32 or t.device != dev:
                    raise ValueError("comm_buffers must be two float32 views of comm_len() on the engine device")
                t.zero_()
        self.params[0][:self.Pimg] = torch.as_tensor(dense_to_image(init_flat, self.dims))
        self.local = self.params[0][:self.Pimg].clone()
        self.mom = torch.zeros(self.Pimg, **f32)
        self.vel = torch.zeros(self.Pimg, **f32)
        sb = self.m.STATE_BYTES
        assert sb == _STATE_DTYPE.itemsize, (sb, _STATE_DTYPE.itemsize)
        init = np.zeros(1, dtype=_STATE_DTYPE)
        init["count"] = cfg.patience
        init["stop_round"] = -1
        st = torch.as_tensor(init.view(np.uint8).copy())
        self.state = [st.to(dev), st.to(dev)]
        if float(cfg.participation) < 1.0 and self.world > 1 and client_sizes is None:
            client_sizes = comm.allgather(self.n_local)
        sched, rtab = self._round_tables(client_sizes)
        self.sched = torch.as_tensor(sched, device=dev)
        self.rtab = torch.as_tensor(rtab, device=dev)
        mr = int(cfg.max_rounds)
        self.h_global = torch.zeros(mr * 4, dtype=torch.float64, device=dev)
        self.h_rank = torch.zeros(mr * self.world * 4, dtype=torch.float64, device=dev)
        self.h_loss = torch.zeros(mr, dtype=torch.float32, device=dev)
        # fp16 gradient slab guard: the Adam kernel sets it when a partial it reads is saturated at
        # +-65504 (slab_store_h's clamp) or not finite; read_history() reports it
        self.sat = torch.zeros(1, dtype=torch.int32, device=dev)
        self.slab_saturated = False
        ecfg = {
            "R": R, "n_rows": self.n_local, "world": self.world, "rank": self.rank, "agg_scale": self.agg_scale,
            "local_steps": int(cfg.local_steps), "lr": float(cfg.lr), "gamma": float(cfg.gamma),
            "step_size": int(cfg.step_size), "beta1": float(cfg.betas[0]), "beta2": float(cfg.betas[1]),
            "eps": float(cfg.eps), "weight_decay": float(cfg.weight_decay), "prox_mu": float(cfg.prox_mu),
            "early_stop": bool(cfg.early_stop), "patience": int(cfg.patience), "atol": float(cfg.tolerance),
            "rtol": float(cfg.rtol), "max_rounds": mr, "metric_mode": _metric_mode_id(cfg.metric_mode),
            "dtype": _dtype_id(cfg.dtype),
            # trial packing runs rounds through run_local + a shared all-reduce: classic rounds
            "fused_eval": bool(cfg.fused_eval) and comm_buffers is None,
            "eval_fedavg": bool(cfg.eval_fedavg),
            "lagged_eval": self._lag,
            "emulate_clients": bool(emulate_clients),
            "slab_f16": self._pick_slab_f16(cfg),
            "plain_fwd": -1 if cfg.plain_fwd is None else int(bool(cfg.plain_fwd)),
        }
        bufs = {
            "X": self.X.data_ptr(), "y": self.y.data_ptr(),
            "local": self.local.data_ptr(), "m": self.mom.data_ptr(), "v": self.vel.data_ptr(),
            "hist_global": self.h_global.data_ptr(), "hist_rank": self.h_rank.data_ptr(),
            "hist_loss": self.h_loss.data_ptr(), "sched": self.sched.data_ptr(), "rtab": self.rtab.data_ptr(),
            "sat": self.sat.data_ptr(),
            "params0": self.params[0].data_ptr(),
            "params1": self.params[1].data_ptr(), "state0": self.state[0].data_ptr(),
            "state1": self.state[1].data_ptr(),
        }
        for i, R in enumerate(R_try):
            self.slab = torch.zeros(((self.n_local + R - 1) // R) * slab_stride, **f32)
            ecfg["R"] = R
            bufs["slab"] = self.slab.data_ptr()
            try:
                self.engine = self.m.FLEngine(self.dims, ecfg, bufs)
                break
            except RuntimeError as err:
                if "LDS" not in str(err) or i + 1 == len(R_try):
                    raise
        self.R = R
        self.layout = self.engine.layout()
        self.slab_f16 = bool(self.layout["slab_f16"])
        iw, ib, _ = image_layout(self.dims)
        if (self.layout["Pimg"], list(self.layout["iw_off"]), list(self.layout["ib_off"])) != (self.Pimg, iw, ib):
            raise RuntimeError(f"image layout mismatch between C++ and Python: {self.layout}")
        # the engine owns a non-default stream: graph capture is illegal on the null stream
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        self.rounds_issued = 0
        self._stopped_seen = False
        self._native_comm = None
        # one-shot xGMI all-reduce of [image | tails] (collective set-up; None -> RCCL)
        self._peer = None
        if self.world > 1 and comm_buffers is None and getattr(comm, "peer_allreduce", False):
            from ..parallel.peer import make_peer_allreduce
            torch.cuda.synchronize(dev)
            # lagged rounds reduce inside the Adam kernel: one chunk flag per Adam block + the
            # two metric-tail chunks
            n_chunks = (self.P + 63) // 64 + 2 if (self._lag and int(cfg.local_steps) == 1) else 0
            self._peer = make_peer_allreduce(comm, comm_len, dev, n_chunks=n_chunks)
            if self._peer is not None:
                self.engine.attach_peer(self._peer)
        if self.world > 1 and self._peer is None and comm_buffers is None and comm is not None \
                and hasattr(comm, "rccl"):
            # RCCL only when the peer plane is off or fell back (every rank agreed on that above),
            # so this lazy, bounded bootstrap runs on every rank or on none; if it fails too, every
            # rank continues on the host plane (aggregation 'host') instead of raising
            self._native_comm = comm.rccl_or_host() if hasattr(comm, "rccl_or_host") else comm.rccl()
        self._graph_ready = False

    def __del__(self):
        # the xGMI communicator's buffers are read by the peers: never freed with the engine, but
        # retired until the next collective set-up (fedmi.parallel.peer.retire)
        peer = getattr(self, "_peer", None)
        if peer is not None:
            try:
                from ..parallel.peer import retire
                retire(peer)
            except Exception:  # noqa: BLE001 -- interpreter shutdown
                pass

    def slab_partials(self) -> torch.Tensor:
        """The last train kernel's per-workgroup gradient partials as [n_slabs, P] (a copy of the
        slab rows, fp32 or fp16, in dense-parameter order).  fp16 partials are sums of the
        unscaled gradient (the Adam kernel applies the 1/n)."""
        lay = self.engine.layout()
        ns, stride, P = int(lay["n_slabs"]), int(lay["slab_stride"]), self.P
        if self.slab_f16:  # fp16 partial e at half e of the row (fl_device.h slab_store_h)
            return self.slab.view(torch.float16).view(-1, 2 * stride)[:ns, :P].clone()
        return self.slab.view(-1, stride)[:ns, :P].clone()

    def _pick_slab_f16(self, cfg) -> bool:
        if cfg.grad_slab not in ("auto", "fp16", "fp32"):
            raise ValueError(f"grad_slab must be 'auto', 'fp16' or 'fp32', got {cfg.grad_slab!r}")
        if cfg.dtype != "bf16" or cfg.grad_slab == "fp32":
            return False
        if cfg.grad_slab == "fp16":
            return True
        if self.X.numel() == 0:
            return True
        lo, hi = torch.aminmax(self.X)  # two scalars, no |X| temporary of the whole shard
        return bool(max(-float(lo), float(hi)) <= FP16_SLAB_MAX_ABS_X)

    def _round_tables(self, client_sizes=None):
        """Host-built device tables (fl_common.h FLBuffers::sched / rtab): per optimizer-step
        slot the Adam/StepLR scalars of this client's own step count (torch's double arithmetic,
        rounded to fp32 once), per round its FedAvg weight and the sampled-client set."""
        cfg = self.cfg
        mr, LS = max(1, int(cfg.max_rounds)), max(1, int(cfg.local_steps))
        b1, b2 = float(cfg.betas[0]), float(cfg.betas[1])
        sched = np.zeros(2 * mr * LS, np.float32)
        scale = np.zeros(mr, np.float32)
        count = np.zeros(mr, np.float32)
        mask = np.zeros((mr, 2), np.uint32)
        t_own = 0
        for r in range(mr):
            part = self.participants(r)
            active = self.rank in part
            if len(part) == self.world:
                w = float(self.n_local) / float(self.n_total)
            else:
                w = float(self.n_local) / float(sum(int(client_sizes[k]) for k in part))
            scale[r] = w if active else 0.0
            count[r] = len(part)
            bits = sum(1 << int(k) for k in part)
            mask[r] = (bits & 0xFFFFFFFF, bits >> 32)
            lr = float(cfg.lr) * float(cfg.gamma) ** (r // int(cfg.step_size))
            for ls in range(LS):
                t_own += int(active)
                t = max(t_own, 1)
                sched[2 * (r * LS + ls)] = lr / (1.0 - b1 ** t)
                sched[2 * (r * LS + ls) + 1] = math.sqrt(1.0 - b2 ** t)
        rtab = np.zeros((mr, 4), np.uint32)
        rtab[:, 0] = scale.view(np.uint32)
        rtab[:, 1] = count.view(np.uint32)
        rtab[:, 2:] = mask
        return sched, rtab.reshape(-1).view(np.int32)

    def _apply_early_stop(self) -> None:
        cfg = self.cfg
        self.engine.set_early_stop(int(cfg.patience), float(cfg.tolerance), float(cfg.rtol))
        self._graph_ready = False
        for st in self.state:     # the patience counter starts at the new patience
            rec = st.cpu().numpy().view(_STATE_DTYPE).copy()
            rec["count"] = int(cfg.patience)
            st.copy_(torch.as_tensor(rec.view(np.uint8)).to(st.device))
        torch.cuda.synchronize(self.device)

    @property
    def aggregation(self) -> str:
        """Data plane of the FedAvg all-reduce: 'none' (one client), 'xgmi-oneshot', 'rccl' or 'host'."""
        if self.world == 1:
            return "none"
        if self._peer is not None:
            return "xgmi-oneshot+adam" if self.engine.adam_exchange else "xgmi-oneshot"
        return "rccl" if self._native_comm is not None else "host"

    # -- execution --
    def _stream(self) -> int:
        return self.stream.cuda_stream

    def _engine_reduces(self) -> bool:
        """The native engine issues the all-reduce itself (peer kernel or RCCL)."""
        return self._peer is not None or self._native_comm is not None

    def _phase_allreduce(self, r: int) -> None:
        if self.world == 1:
            return
        if self._engine_reduces():
            self.engine.phase(r, 2, self._stream(), self._native_comm)
        else:
            with torch.cuda.stream(self.stream):
                self.comm.allreduce_(self.params[(r + 1) & 1])

    def _issue_debug(self, n: int) -> None:
        """Debug mode: every phase launched eagerly and synchronised, so a
        fault is attributed to its kernel, and weights / metric tails checked for NaN/Inf
        after every local step and every aggregation."""
        s = self._stream()
        for _ in range(n):
            r = self.rounds_issued
            out = self.params[(r + 1) & 1]
            self.engine.phase(r, 0, s, None)
            self.stream.synchronize()
            _check_finite(r, "local weights after the Adam step", self.local)
            self.engine.phase(r, 1, s, None)
            self.stream.synchronize()
            self._phase_allreduce(r)
            self.stream.synchronize()
            _check_finite(r, "aggregated weights / metric tails", out)
            self.rounds_issued += 1

    def profile(self, n: int) -> Dict[str, float]:
        """Run ``n`` live rounds eagerly with hipEvents around each phase; returns mean
        microseconds of local step (train + Adam kernels), eval, all-reduce and round."""
        s = self._stream()
        names = ("train", "eval", "allreduce")
        acc = dict.fromkeys(names + ("round",), 0.0)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        n = min(n, self.cfg.max_rounds - self.rounds_issued)
        for _ in range(n):
            r = self.rounds_issued
            ev[0].record(self.stream)
            self.engine.phase(r, 0, s, None)
            ev[1].record(self.stream)
            self.engine.phase(r, 1, s, None)
            ev[2].record(self.stream)
            self._phase_allreduce(r)
            ev[3].record(self.stream)
            self.stream.synchronize()
            for i, k in enumerate(names):
                acc[k] += 1e3 * ev[i].elapsed_time(ev[i + 1])
            acc["round"] += 1e3 * ev[0].elapsed_time(ev[3])
            self.rounds_issued += 1
        self.sync_history()
        return {k + "_us": v / max(n, 1) for k, v in acc.items()}

    def trace(self, n: int, close: bool = False, gate_us: float = 5000.0, warm: int = 0) -> Dict[str, object]:
        """Per-kernel breakdown of ``n`` rounds of the engine's REAL round design (unlike
        :meth:`profile`, which runs classic phases): the native engine issues them eagerly with
        a hipEvent after every launch behind a gate kernel (FLEngine::trace), so the kernels
        run back to back.  Returns mean us per round by kernel kind (``train``, ``adam``,
        ``eval``, ``pack``, ``allreduce``, ``eval_fedavg``), ``round`` and launch counts.  Each
        interval carries the eager launch + event marker cost: measured on MI355X (bench N = 1,
        profiles/kernel_trace_r5.log) ~1.5 us per kernel over the rocprofv3 kernel durations
        (markers without the system-scope fence; ~3.2 us with it).
        Collective on multi-client engines (every rank must call it with the same ``n``);
        ``warm`` untraced rounds run first behind the gate (they absorb the ranks' start skew)."""
        if self.cfg.debug or (self.world > 1 and not self._engine_reduces()):
            raise RuntimeError("trace: needs an engine that issues its own FedAvg")
        n, warm = int(n), int(warm)
        if n < 1 or warm < 0 or self.rounds_issued + warm + n > self.cfg.max_rounds:
            raise RuntimeError("trace: needs n >= 1 and warm + n rounds left (max_rounds)")
        # (pending host-side weight changes etc. are handled inside run(), like eager rounds)
        out = dict(self.engine.trace(self.rounds_issued, n, self._stream(), self._native_comm,
                                     close=close, gate_us=gate_us, warm=warm))
        self.rounds_issued += warm + n
        return out

    def _issue(self, n: int, close: bool = True, graph_rounds: Optional[int] = None) -> None:
        """Issue rounds [rounds_issued, rounds_issued + n) on the current stream.

        ``close=False`` (lagged engines): the last round stays lagged -- its evaluation is
        done by the next issued round's train kernel, so every round of the call can be a
        graph replay.  The host must issue at least one more (closing) round before it reads
        the history.  ``graph_rounds``: rounds per replayed graph (default: the config's)."""
        if self.cfg.debug:
            self._issue_debug(n)
            return
        s = self._stream()
        r0 = self.rounds_issued
        g = int(self.cfg.graph_rounds if graph_rounds is None else graph_rounds)
        if self.world > 1 and not self._engine_reduces():
            # torch-owned communicator: all-reduce from Python between rounds
            with torch.cuda.stream(self.stream):
                for r in range(r0, r0 + n):
                    self.engine.run_local(r, s)
                    self.comm.allreduce_(self.params[(r + 1) & 1])
            self.rounds_issued += n
            return
        # lagged engines: graphs hold lagged rounds only, the last round of the call is eager and
        # evaluates itself (then every metric is in the buffers for the host)
        lag = bool(self.engine.lagged) and close
        r = r0
        while r < r0 + n:
            left = r0 + n - r
            if (g >= 2 and r % 2 == 0 and (left > g if lag else left >= g)
                    and not self.engine.needs_eager_round()):
                self._ensure_graph(g)
                self.engine.replay(s)
                r += g
            else:
                self.engine.run(r, 1, s, self._native_comm, close=(close and r == r0 + n - 1))
                r += 1
        self.rounds_issued = r

    def set_debug(self, ptr: int) -> None:
        """Phase stamps (fl_device.h) into the device buffer at ``ptr`` (0: off).  A configuration
        change: the native engine drops its cached graphs, and so does this side."""
        self.engine.set_debug(int(ptr))
        self._graph_ready = False

    def _ensure_graph(self, g: int) -> None:
        if not self._graph_ready or self.engine.graph_rounds() != g:
            self.engine.capture(g, self._stream(), self._native_comm)
            self._graph_ready = True

    def prime_graph(self, g: int, replays: int = 1) -> int:
        """Bring the engine to the steady state of a ``g``-round graph before a timed region:
        issue (uncounted by the caller) eager rounds until the next round is even and may start
        a graph, capture + instantiate the graph and replay it ``replays`` times (the second launch
        of a freshly instantiated graph runs ~0.6 us per round slower than later ones,
        profiles/short_region_r4*.log).  Afterwards ``_issue(k * g, close=False)`` is ``k`` graph
        replays.  Returns the rounds issued."""
        if g < 2 or g % 2:
            raise ValueError("graph rounds must be an even number >= 2")
        if self.world > 1 and not self._engine_reduces():
            raise RuntimeError("prime_graph: rounds aggregated from Python are not captured")
        self.cfg.graph_rounds = g
        r0 = self.rounds_issued
        s = self._stream()
        for _ in range(4):
            if self.rounds_issued % 2 == 0 and not self.engine.needs_eager_round():
                break
            self.engine.run(self.rounds_issued, 1, s, self._native_comm, close=False)
            self.rounds_issued += 1
        else:
            raise RuntimeError("prime_graph: engine did not reach a graph-capturable state")
        self._ensure_graph(g)
        for _ in range(max(1, int(replays))):
            self.engine.replay(s)
            self.rounds_issued += g
        return self.rounds_issued - r0

    def _read_state(self, idx: int) -> np.ndarray:
        self.stream.synchronize()
        self._check_peer()
        return self.state[idx].cpu().numpy().view(_STATE_DTYPE)[0]

    # -- step-by-step API (reference train_one_epoch / evaluate_local / federated_averaging)
    def step_train(self) -> None:
        self.engine.phase(self.rounds_issued, 0, self._stream(), None)

    def step_eval(self) -> np.ndarray:
        r = self.rounds_issued
        self.engine.phase(r, 1, self._stream(), None)
        self.stream.synchronize()
        C = self.n_classes
        t0 = self.Pimg + self.rank * self.tail_stride
        if self._peer is not None:  # published into the peer send buffer, not yet reduced
            cm = np.asarray(self._peer.read((r + 1) & 1, t0, C * C), dtype=np.float32)
        else:
            cm = self.params[(r + 1) & 1][t0:t0 + C * C].cpu().numpy()
        return cm.reshape(C, C).astype(np.int64)

    def step_aggregate(self) -> None:
        r = self.rounds_issued
        self._phase_allreduce(r)
        self.rounds_issued += 1
        st = self._read_state(self.rounds_issued & 1)
        if st["stopped"]:
            self._stopped_seen = True

    def run(self, n_rounds: int, check_every: int = 64) -> int:
        """Run up to ``n_rounds`` rounds; returns the number of live rounds.  The stop
        flag is polled once per ``check_every`` rounds (rounds issued past an early stop
        are exact no-ops on the device)."""
        before = self.hist.rounds_run
        left = min(n_rounds, self.cfg.max_rounds - self.rounds_issued)
        while left > 0 and not self._stopped_seen:
            n = min(left, check_every)
            self._issue(n)
            left -= n
            st = self._read_state(self.rounds_issued & 1)
            if st["stopped"]:
                self._stopped_seen = True
        self.sync_history()
        return self.hist.rounds_run - before

    def run_streaming(self, n_rounds: int, chunk: int = 16, on_history=None, guard=None) -> int:
        """:meth:`run` with the metrics streamed as the rounds complete: rounds are issued in
        chunks of ``chunk``, and after each chunk a finalize plus an asynchronous copy of the
        round state and metric history into pinned host memory are queued behind it.  Chunk k+1
        is issued BEFORE chunk k's copy is waited on, so the device never idles on the host, and
        ``on_history(history)`` sees round r while at most one chunk (<= ``chunk`` rounds) runs
        after it (the reference prints every round as it completes, C:139-179).  ``guard(desc)``:
        optional context manager around each chunk (the collective watchdog).  Returns the number
        of live rounds; rounds issued past an early stop are exact no-ops on the device."""
        import contextlib
        before = self.hist.rounds_run
        left = min(int(n_rounds), self.cfg.max_rounds - self.rounds_issued)
        if self.cfg.debug or (self.world > 1 and not self._engine_reduces()):
            while left > 0 and not self._stopped_seen:   # host-driven rounds: chunk by chunk
                n = min(chunk, left)
                with (guard(f"rounds {self.rounds_issued}..{self.rounds_issued + n - 1}") if guard
                      else contextlib.nullcontext()):
                    self.run(n, check_every=n)
                left -= n
                if on_history is not None:
                    on_history(self.history())
            return self.hist.rounds_run - before
        # graph rounds per chunk: lagged engines close every chunk with an eager self-evaluating
        # round, and a lagged graph starts only behind a lagged round that scored its predecessor
        # (FLEngine::needs_eager_round), so a chunk is 2 eager lagged rounds + the graph + 1 lagged
        # + the closing round (graph + 4, even, so every chunk starts on an even round)
        g = int(self.cfg.graph_rounds)
        if g >= 2:
            gs = max(2, (min(g, chunk) - (4 if self.engine.lagged else 0)) & ~1)
            step = gs + (4 if self.engine.lagged else 0)
        else:
            gs, step = 0, max(1, chunk)
        mirror = self._host_mirror()
        s = self._stream()
        pend = None
        slot = 0
        while True:
            new = None
            if left > 0 and not self._stopped_seen:
                n = min(step, left)
                desc = f"rounds {self.rounds_issued}..{self.rounds_issued + n - 1}"
                with (guard(desc) if guard else contextlib.nullcontext()):
                    self._issue(n, graph_rounds=gs)
                left -= n
                r = self.rounds_issued
                self.engine.finalize(r, s)
                m = mirror[slot]
                with torch.cuda.stream(self.stream):
                    m["state"].copy_(self.state[(r + 1) & 1], non_blocking=True)
                    m["glob"].copy_(self.h_global, non_blocking=True)
                    m["rank"].copy_(self.h_rank, non_blocking=True)
                    m["loss"].copy_(self.h_loss, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
                new = (ev, slot, desc)
                slot ^= 1
            if pend is not None:
                with (guard(pend[2]) if guard else contextlib.nullcontext()):
                    pend[0].synchronize()
                # fail fast: a failure reported on the xGMI plane (a peer died / stalled, or
                # aborted) invalidates this chunk's rounds -- raise before they are folded or printed
                self._check_peer()
                self._fold_mirror(mirror[pend[1]])
                if on_history is not None:
                    on_history(self.history())
            pend = new
            if pend is None:
                break
        self._check_peer()
        self._check_slab_saturation()
        return self.hist.rounds_run - before

    def _check_peer(self) -> None:
        """Raise (fedmi.parallel.peer.PeerFailure) if any rank reported a failure of the xGMI
        data plane; every host-visible result since then is invalid."""
        if self._peer is not None:
            from ..parallel.peer import check_peer_error
            check_peer_error(self._peer)

    def _host_mirror(self):
        """Two pinned-host copies (double-buffered by chunk) of the round state and history."""
        if getattr(self, "_mirror", None) is None:
            pin = torch.cuda.is_available()
            mk = lambda t: torch.empty(t.shape, dtype=t.dtype, pin_memory=pin)
            self._mirror = [{"state": mk(self.state[0]), "glob": mk(self.h_global), "rank": mk(self.h_rank),
                             "loss": mk(self.h_loss)} for _ in range(2)]
        return self._mirror

    def _fold_mirror(self, m) -> None:
        st = m["state"].numpy().view(_STATE_DTYPE)[0]
        n = int(st["finalized"])
        self.hist.rounds_run = n
        if n:
            self.hist.glob[:n] = m["glob"][:n * 4].numpy().reshape(n, 4)
            self.hist.rank[:n] = m["rank"][:n * self.world * 4].numpy().reshape(n, self.world, 4)
            self.hist.loss[:n] = m["loss"][:n].numpy()
        if st["stopped"]:
            self.hist.stop_round = int(st["stop_round"])
            self.hist.stop_trigger = int(st["stop_round"]) - 1
            self._stopped_seen = True

    @property
    def stopped(self) -> bool:
        return self._stopped_seen

    def sync_history(self) -> None:
        r = self.rounds_issued
        s = self._stream()
        self.engine.finalize(r, s)
        self.read_history()

    def read_history(self) -> None:
        """Copy the device history of the rounds issued into ``hist`` (after a finalize of
        ``rounds_issued``: this engine's ``sync_history`` or its trial batch's)."""
        r = self.rounds_issued
        st = self._read_state((r + 1) & 1)   # synchronizes the engine stream
        n = int(st["finalized"])
        self.hist.rounds_run = n
        if n:
            self.hist.glob[:n] = self.h_global[:n * 4].cpu().numpy().reshape(n, 4)
            self.hist.rank[:n] = self.h_rank[:n * self.world * 4].cpu().numpy().reshape(n, self.world, 4)
            self.hist.loss[:n] = self.h_loss[:n].cpu().numpy()
        if st["stopped"]:
            self.hist.stop_round = int(st["stop_round"])
            self.hist.stop_trigger = int(st["stop_round"]) - 1
            self._stopped_seen = True
        self._check_slab_saturation()

    def _check_slab_saturation(self) -> None:
        if self.slab_f16 and not self.slab_saturated and int(self.sat.item()):
            self.slab_saturated = True
            msg = ("fp16 gradient slab saturated (a per-workgroup partial reached +-65504 or is not finite): the "
                   "gradients of those rounds are clipped; rerun with EngineConfig(grad_slab='fp32')")
            if self.cfg.debug:
                raise FloatingPointError(msg)
            import warnings
            warnings.warn(msg, RuntimeWarning, stacklevel=2)

    def global_flat(self) -> np.ndarray:
        self.stream.synchronize()
        return image_to_dense(self.params[self.rounds_issued & 1][:self.Pimg].cpu().numpy(), self.dims)

    def local_flat(self) -> np.ndarray:
        self.stream.synchronize()
        return image_to_dense(self.local.cpu().numpy(), self.dims)

    def set_global_flat(self, flat: np.ndarray) -> None:
        self.stream.synchronize()
        self.params[self.rounds_issued & 1][:self.Pimg].copy_(torch.as_tensor(dense_to_image(flat, self.dims)))
        torch.cuda.current_stream(self.device).synchronize()
        self.engine.invalidate()

    def confusion(self, X=None, y=None, flat=None) -> np.ndarray:
        Xt = self.X if X is None else torch.as_tensor(np.ascontiguousarray(X, np.float32), device=self.device)
        yt = self.y if y is None else torch.as_tensor(np.asarray(y), dtype=torch.int32, device=self.device)
        if flat is None:
            p = self.local
        else:
            p = torch.as_tensor(dense_to_image(flat, self.dims), device=self.device)
        cm = torch.zeros(self.n_classes ** 2, dtype=torch.float32, device=self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.engine.confusion(Xt.data_ptr(), yt.data_ptr(), int(Xt.shape[0]), p.data_ptr(), cm.data_ptr(),
                              self._stream())
        self.stream.synchronize()
        return cm.cpu().numpy().reshape(self.n_classes, self.n_classes).astype(np.int64)

    def portable_state(self) -> dict:
        self.sync_history()
        r = self.rounds_issued
        st = self._read_state((r + 1) & 1)   # the finalized copy (sync_history folded round r-1)
        return {
            "rounds": int(r), "global": self.global_flat(), "local": self.local_flat(),
            "exp_avg": image_to_dense(self.mom.cpu().numpy(), self.dims),
            "exp_avg_sq": image_to_dense(self.vel.cpu().numpy(), self.dims), "opt_steps": self.own_steps(int(r)),
            "es": {"count": int(st["count"]), "has_prev": bool(st["has_prev"]),
                   "prev": [float(x) for x in st["prev"]], "stopped": bool(st["stopped"]),
                   "stop_round": int(st["stop_round"])},
            "history": self.hist.as_dict(),
        }

    def load_portable_state(self, st: dict) -> None:
        r = int(st["rounds"])
        if r > self.cfg.max_rounds:
            raise ValueError(f"checkpoint has {r} rounds > max_rounds {self.cfg.max_rounds}")
        self.stream.synchronize()
        dev = self.device
        img = lambda a: torch.as_tensor(dense_to_image(np.asarray(a, np.float32), self.dims), device=dev)
        with torch.cuda.stream(self.stream):
            self.params[r & 1][:self.Pimg].copy_(img(st["global"]))
            self.local.copy_(img(st["local"]))
            self.mom.copy_(img(st["exp_avg"]))
            self.vel.copy_(img(st["exp_avg_sq"]))
            es = st["es"]
            rec = np.zeros(1, dtype=_STATE_DTYPE)
            rec["next_round"] = r
            rec["finalized"] = r
            rec["cur_round"] = r - 1
            rec["count"] = int(es["count"])
            rec["has_prev"] = int(bool(es["has_prev"]))
            rec["prev"] = np.asarray(es["prev"], np.float64)
            rec["stopped"] = int(bool(es["stopped"]))
            rec["stop_round"] = int(es["stop_round"])
            # the peer exchange's call counter stays monotonic (peers' flags hold past calls)
            rec["calls"] = max(int(self.state[q].cpu().numpy().view(_STATE_DTYPE)[0]["calls"]) for q in (0, 1))
            self.state[r & 1].copy_(torch.as_tensor(rec.view(np.uint8).copy()).to(dev))
            self._load_history(st["history"])
            n = self.hist.rounds_run
            if n:
                self.h_global[:n * 4].copy_(torch.as_tensor(self.hist.glob[:n].reshape(-1), device=dev))
                self.h_rank[:n * self.world * 4].copy_(torch.as_tensor(self.hist.rank[:n].reshape(-1), device=dev))
                self.h_loss[:n].copy_(torch.as_tensor(self.hist.loss[:n], device=dev))
        self.stream.synchronize()
        self.engine.invalidate()
        self.engine.reset_pending()
        self.rounds_issued = r
        self._stopped_seen = bool(st["es"]["stopped"])

    def state_dict(self) -> dict:
        self.stream.synchronize()
        return {"params": self.global_flat(), "local": self.local_flat(),
                "exp_avg": image_to_dense(self.mom.cpu().numpy(), self.dims),
                "exp_avg_sq": image_to_dense(self.vel.cpu().numpy(), self.dims), "rounds": self.rounds_issued,
                "state": self.state[self.rounds_issued & 1].cpu().numpy(), "history": self.hist.as_dict()}


def _check_finite(r: int, what: str, t: torch.Tensor) -> None:
    if not bool(torch.isfinite(t).all()):
        bad = int((~torch.isfinite(t)).sum())
        raise FloatingPointError(f"round {r}: {bad} non-finite values in {what}")


def comm_len(dims: Sequence[int], world: int) -> int:
    """Floats in one FedAvg buffer of the HIP engine: parameter image + per-rank tails."""
    n_classes = int(dims[-1])
    return image_layout(list(dims))[2] + world * (n_classes * n_classes + 1)


class _ShapeOnly:
    """Stand-in so the base class can read ``len(X)``/``X.shape`` of device tensors."""

    def __init__(self, n, f):
        self.shape = (n, f)

    def __len__(self):
        return self.shape[0]


def make_engine(X, y, n_classes, cfg: EngineConfig, comm, init_flat, n_total=None, backend: str = "auto"):
    if backend == "auto":
        backend = "hip" if (comm is not None and comm.device.type == "cuda") or \
            (comm is None and torch.cuda.is_available()) else "torch"
    if backend == "hip":
        return HipRoundEngine(X, y, n_classes, cfg, comm, init_flat, n_total)
    if backend == "torch":
        return TorchRoundEngine(X, y, n_classes, cfg, comm, init_flat, n_total)
    raise ValueError(f"unknown engine backend {backend!r}")
