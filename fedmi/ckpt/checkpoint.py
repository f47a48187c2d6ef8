"""Checkpoint / resume in the reference's weight-exchange layout.

The reference persists nothing; its de-facto checkpoint layout is the in-memory exchange
format: the ``named_parameters()`` dict ``model.{2i}.weight`` [out, in] /
``model.{2i}.bias`` fp32 ([C], C:93-94) and, for sklearn, ``coefs_ + intercepts_``
([in, out], float64; S:26).  A fedmi checkpoint is a directory with

* ``weights.safetensors``       -- the global (aggregated) model under the reference key
  names, loadable into a plain ``torch.nn`` model of the reference with ``load_state_dict``;
* ``client{r}.safetensors``     -- per client r: local weights, the flat Adam
  ``exp_avg`` / ``exp_avg_sq`` (they persist across rounds in the reference, Q6) and the
  client's own Adam step count (client sampling: a client only steps when sampled);
* ``meta.json``                 -- dims, rounds done (= StepLR counter and Adam step),
  engine config, replicated early-stop state and the metric history.

Only safetensors / JSON: nothing in a checkpoint can execute code on load.  The state is
engine-independent (dense reference layout), so a run checkpointed on the HIP engine
resumes on the torch engine and vice versa.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

import numpy as np

from ..models.mlp import dict_to_flat, flat_to_dict

FORMAT = "fedmi-ckpt-2"


def _st():
    from safetensors.numpy import load_file, save_file
    return save_file, load_file


def save_weights(path: str, weights: Dict[str, np.ndarray]) -> None:
    save_file, _ = _st()
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()}, path)


def load_weights(path: str) -> Dict[str, np.ndarray]:
    _, load_file = _st()
    return dict(load_file(path))


def _engine(obj):
    """Round engine of a trainer (``FederatedMLPLearning.engine``) or the engine itself."""
    return obj if hasattr(obj, "portable_state") else obj.engine


def _barrier(eng) -> None:
    comm = getattr(eng, "comm", None)
    if comm is not None and getattr(comm, "size", 1) > 1:
        comm.Barrier()


def save_checkpoint(path: str, trainer) -> None:
    """Collective over the clients: every rank writes its own ``client{r}`` file, rank 0
    writes the global weights and the metadata."""
    eng = _engine(trainer)
    st = eng.portable_state()
    os.makedirs(path, exist_ok=True)
    save_file, _ = _st()
    save_file({"local": np.asarray(st["local"], np.float32), "exp_avg": np.asarray(st["exp_avg"], np.float32),
               "exp_avg_sq": np.asarray(st["exp_avg_sq"], np.float32),
               # this client's own Adam step count (differs from rounds x local_steps when clients are sampled)
               "opt_steps": np.asarray([int(st.get("opt_steps", 0))], np.int64)},
              os.path.join(path, f"client{eng.rank}.safetensors"))
    if eng.rank == 0:
        save_weights(os.path.join(path, "weights.safetensors"), flat_to_dict(st["global"], eng.dims))
        hist = st["history"]
        meta = {
            "format": FORMAT,
            "dims": list(eng.dims),
            "rounds": int(st["rounds"]),
            "config": eng.cfg.to_dict(),
            "world": eng.world,
            "early_stop": st["es"],
            "history": {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in hist.items()},
        }
        tmp = os.path.join(path, "meta.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f)
        os.replace(tmp, os.path.join(path, "meta.json"))
    _barrier(eng)


def load_checkpoint(path: str, rank: Optional[int] = None) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: unsupported checkpoint format {meta.get('format')!r}")
    w = load_weights(os.path.join(path, "weights.safetensors"))
    out = {"meta": meta, "weights": w, "flat": dict_to_flat(w, meta["dims"])}
    if rank is not None:
        cp = os.path.join(path, f"client{rank}.safetensors")
        if os.path.isfile(cp):
            _, load_file = _st()
            out["client"] = dict(load_file(cp))
    return out


def resume(path: str, trainer) -> int:
    """Restore a run saved by :func:`save_checkpoint` into ``trainer`` (same dims and
    client count); returns the number of rounds already done."""
    eng = _engine(trainer)
    ck = load_checkpoint(path, rank=eng.rank)
    meta = ck["meta"]
    if list(meta["dims"]) != list(eng.dims):
        raise ValueError(f"checkpoint dims {meta['dims']} != model dims {eng.dims}")
    if int(meta["world"]) != eng.world:
        raise ValueError(f"checkpoint has {meta['world']} clients, this run has {eng.world}")
    if "client" not in ck:
        raise FileNotFoundError(f"{path}: no client{eng.rank}.safetensors")
    c = ck["client"]
    h = meta["history"]
    st = {"rounds": int(meta["rounds"]), "global": ck["flat"], "local": c["local"], "exp_avg": c["exp_avg"],
          "exp_avg_sq": c["exp_avg_sq"], "es": meta["early_stop"],
          "history": {"rounds_run": h["rounds_run"], "stop_round": h["stop_round"],
                      "stop_trigger": h["stop_trigger"], "global": np.asarray(h["global"]),
                      "per_rank": np.asarray(h["per_rank"]), "loss": np.asarray(h["loss"])}}
    if "opt_steps" in c:
        st["opt_steps"] = int(np.asarray(c["opt_steps"]).reshape(-1)[0])
    eng.load_portable_state(st)
    return st["rounds"]


# ---------------------------------------------------------------------------------------
# sklearn layout ([S] / [H] flows): the exchange list coefs_ + intercepts_ (S:26, S:109, H:30)
# ---------------------------------------------------------------------------------------
SK_FORMAT = "fedmi-sklearn-ckpt-1"


def save_sklearn_weights(path: str, weights) -> None:
    """``weights`` = the reference's flat exchange list ``coefs_ + intercepts_``: L coefficient
    matrices [in, out] then L intercept vectors, float64 (S:26).  Stored as safetensors keys
    ``coefs_.{i}`` / ``intercepts_.{i}``, float64, same shapes."""
    save_file, _ = _st()
    ws = [np.asarray(w, dtype=np.float64) for w in weights]
    L = len(ws) // 2
    if len(ws) != 2 * L or any(ws[i].ndim != 2 or ws[L + i].shape != (ws[i].shape[1],) for i in range(L)):
        raise ValueError("expected coefs_ ([in, out] matrices) followed by intercepts_ ([out] vectors)")
    t = {f"coefs_.{i}": np.ascontiguousarray(ws[i]) for i in range(L)}
    t.update({f"intercepts_.{i}": np.ascontiguousarray(ws[L + i]) for i in range(L)})
    save_file(t, path)


def load_sklearn_weights(path: str):
    """Inverse of :func:`save_sklearn_weights`: the ``coefs_ + intercepts_`` list, float64."""
    _, load_file = _st()
    t = dict(load_file(path))
    L = sum(1 for k in t if k.startswith("coefs_."))
    if L == 0 or any(f"coefs_.{i}" not in t or f"intercepts_.{i}" not in t for i in range(L)):
        raise ValueError(f"{path}: not a coefs_/intercepts_ checkpoint")
    return [t[f"coefs_.{i}"] for i in range(L)] + [t[f"intercepts_.{i}"] for i in range(L)]


def sklearn_to_torch_layout(weights):
    """coefs_ + intercepts_ ([in, out]) -> the [C] ``model.{2i}.weight`` [out, in] / ``.bias`` dict."""
    L = len(weights) // 2
    out = {}
    for i in range(L):
        out[f"model.{2 * i}.weight"] = np.ascontiguousarray(np.asarray(weights[i]).T, dtype=np.float32)
        out[f"model.{2 * i}.bias"] = np.asarray(weights[L + i], dtype=np.float32)
    return out


def save_sklearn_run(path: str, rank: int, round_done: int, global_weights, local_weights, meta: dict,
                     comm=None) -> None:
    """[S] round checkpoint (collective): rank 0 writes ``global.safetensors`` + ``meta.json``
    (rounds done, history, run settings), every rank its local model ``client{r}.safetensors``.
    Every file is written to a temporary name and renamed into place, and ``meta.json`` -- the
    file that says which round the directory holds -- is written LAST, after a barrier: a crash
    at any point leaves either the previous round's complete set or the new one."""
    os.makedirs(path, exist_ok=True)

    def _atomic_weights(name, w):
        tmp = os.path.join(path, f".{name}.tmp{os.getpid()}")
        save_sklearn_weights(tmp, w)
        os.replace(tmp, os.path.join(path, name))

    _atomic_weights(f"client{rank}.safetensors", local_weights)
    if rank == 0 and global_weights is not None:
        _atomic_weights("global.safetensors", global_weights)
    if comm is not None and getattr(comm, "size", 1) > 1:
        comm.Barrier()   # every client file of this round is in place
    if rank == 0:
        m = dict(meta, format=SK_FORMAT, rounds=int(round_done))
        tmp = os.path.join(path, "meta.json.tmp")
        with open(tmp, "w") as f:
            json.dump(m, f)
        os.replace(tmp, os.path.join(path, "meta.json"))
    if comm is not None and getattr(comm, "size", 1) > 1:
        comm.Barrier()   # nobody reads / rewrites the directory before meta.json points at it


def load_sklearn_run(path: str, rank: int) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != SK_FORMAT:
        raise ValueError(f"{path}: unsupported checkpoint format {meta.get('format')!r}")
    out = {"meta": meta, "local": load_sklearn_weights(os.path.join(path, f"client{rank}.safetensors"))}
    gp = os.path.join(path, "global.safetensors")
    out["global"] = load_sklearn_weights(gp) if os.path.isfile(gp) else None
    return out
