"""Checkpoint / resume in the reference's weight-exchange layout.

The reference persists nothing; its de-facto checkpoint layout is the in-memory exchange
format: the ``named_parameters()`` dict ``model.{2i}.weight`` [out, in] /
``model.{2i}.bias`` fp32 ([C], C:93-94) and, for sklearn, ``coefs_ + intercepts_``
([in, out], float64; S:26).  A fedmi checkpoint is a directory with

* ``weights.r<R>.safetensors``  -- the global (aggregated) model of round R under the reference
  key names, loadable into a plain ``torch.nn`` model of the reference with ``load_state_dict``
  (``weights.safetensors``: a convenience copy of the latest);
* ``client{r}.r<R>.safetensors`` -- per client r: local weights, the flat Adam
  ``exp_avg`` / ``exp_avg_sq`` (they persist across rounds in the reference, Q6) and the
  client's own Adam step count (client sampling: a client only steps when sampled);
* ``meta.json``                 -- dims, rounds done (= StepLR counter and Adam step), the
  names of the round's files, engine config, replicated early-stop state and the metric
  history.  Written last: it is what makes a round's set the checkpoint (see ``tagged``).

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

FORMAT = "fedmi-ckpt-3"
_OLD_FORMATS = ("fedmi-ckpt-2",)   # untagged file names; still loadable


def _st():
    from safetensors.numpy import load_file, save_file
    return save_file, load_file


def save_weights(path: str, weights: Dict[str, np.ndarray], rounds: Optional[int] = None) -> None:
    save_file, _ = _st()
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()}, path,
              metadata=None if rounds is None else {"round": str(int(rounds))})


def load_weights(path: str, expect_round: Optional[int] = None) -> Dict[str, np.ndarray]:
    _, load_file = _st()
    _check_round(path, expect_round)
    return dict(load_file(path))


# ---------------------------------------------------------------------------------------
# Round-tagged file sets.  A checkpoint directory holds, per saved round R, files named
# ``<stem>.r<R>.safetensors`` whose safetensors header records R; ``meta.json`` -- written last,
# atomically, after a barrier -- names the round and hence the set.  A crash anywhere leaves the
# previous meta.json pointing at the previous round's complete set (its files are pruned only
# after the new meta.json is in place), and a loader rejects a file whose header round differs
# from meta.json's (no mixing of weights from different rounds).
# ---------------------------------------------------------------------------------------
def tagged(name: str, rounds: int) -> str:
    """``client0.safetensors`` -> ``client0.r12.safetensors``."""
    stem, ext = name.rsplit(".", 1)
    return f"{stem}.r{int(rounds)}.{ext}"


def _atomic(path: str, write) -> None:
    d, base = os.path.split(path)
    tmp = os.path.join(d, f".{base}.tmp{os.getpid()}")
    write(tmp)
    os.replace(tmp, path)


def _publish_meta(dirpath: str, meta: dict, name: str = "meta.json") -> None:
    def w(tmp):
        with open(tmp, "w") as f:
            json.dump(meta, f)
            f.flush()
            os.fsync(f.fileno())
    _atomic(os.path.join(dirpath, name), w)


def _check_round(path: str, expect_round: Optional[int]) -> None:
    if expect_round is None:
        return
    from safetensors import safe_open
    with safe_open(path, framework="numpy") as f:
        md = f.metadata() or {}
    if "round" not in md or int(md["round"]) != int(expect_round):
        raise ValueError(f"{path}: holds round {md.get('round')!r}, the checkpoint's meta.json says {expect_round}")


def _prune(dirpath: str, name: str, keep_round: int) -> None:
    """Remove this file's round-tagged copies other than ``keep_round`` (and a legacy untagged
    copy): called after meta.json points at ``keep_round``."""
    stem, ext = name.rsplit(".", 1)
    keep = tagged(name, keep_round)
    for f in os.listdir(dirpath):
        if f == keep or not f.startswith(stem + ".r") or not f.endswith("." + ext):
            continue
        mid = f[len(stem) + 2:-(len(ext) + 1)]
        if mid.isdigit():
            try:
                os.remove(os.path.join(dirpath, f))
            except FileNotFoundError:
                pass


def _engine(obj):
    """Round engine of a trainer (``FederatedMLPLearning.engine``) or the engine itself."""
    return obj if hasattr(obj, "portable_state") else obj.engine


def _barrier(eng) -> None:
    comm = getattr(eng, "comm", None)
    if comm is not None and getattr(comm, "size", 1) > 1:
        comm.Barrier()


def save_checkpoint(path: str, trainer) -> None:
    """Collective over the clients: every rank writes its own ``client{r}`` file, rank 0
    writes the global weights and, after a barrier, the metadata that names the round's set.
    ``weights.safetensors`` (untagged) is refreshed afterwards as a convenience copy of the
    global model in the reference layout."""
    eng = _engine(trainer)
    st = eng.portable_state()
    R = int(st["rounds"])
    os.makedirs(path, exist_ok=True)
    save_file, _ = _st()
    cname = f"client{eng.rank}.safetensors"
    _atomic(os.path.join(path, tagged(cname, R)), lambda tmp: save_file(
        {"local": np.asarray(st["local"], np.float32), "exp_avg": np.asarray(st["exp_avg"], np.float32),
         "exp_avg_sq": np.asarray(st["exp_avg_sq"], np.float32),
         # this client's own Adam step count (differs from rounds x local_steps when clients are sampled)
         "opt_steps": np.asarray([int(st.get("opt_steps", 0))], np.int64)}, tmp, metadata={"round": str(R)}))
    gflat = flat_to_dict(st["global"], eng.dims)
    if eng.rank == 0:
        _atomic(os.path.join(path, tagged("weights.safetensors", R)), lambda tmp: save_weights(tmp, gflat, R))
    _barrier(eng)   # every file of round R is in place
    if eng.rank == 0:
        hist = st["history"]
        _publish_meta(path, {
            "format": FORMAT,
            "dims": list(eng.dims),
            "rounds": R,
            "files": {"weights": tagged("weights.safetensors", R), "client": tagged("client{rank}.safetensors", R)},
            "config": eng.cfg.to_dict(),
            "world": eng.world,
            "early_stop": st["es"],
            "history": {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in hist.items()},
        })
    _barrier(eng)   # meta.json names round R: older sets may go
    _prune(path, cname, R)
    if eng.rank == 0:
        _prune(path, "weights.safetensors", R)
        _atomic(os.path.join(path, "weights.safetensors"), lambda tmp: save_weights(tmp, gflat, R))


def load_checkpoint(path: str, rank: Optional[int] = None) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    fmt = meta.get("format")
    if fmt != FORMAT and fmt not in _OLD_FORMATS:
        raise ValueError(f"{path}: unsupported checkpoint format {fmt!r}")
    R = int(meta["rounds"]) if fmt == FORMAT else None
    files = meta.get("files", {"weights": "weights.safetensors", "client": "client{rank}.safetensors"})
    w = load_weights(os.path.join(path, files["weights"]), expect_round=R)
    out = {"meta": meta, "weights": w, "flat": dict_to_flat(w, meta["dims"])}
    if rank is not None:
        cp = os.path.join(path, files["client"].format(rank=rank))
        if os.path.isfile(cp):
            _, load_file = _st()
            _check_round(cp, R)
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
        raise FileNotFoundError(f"{path}: no client file for rank {eng.rank} (round {meta['rounds']})")
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
SK_FORMAT = "fedmi-sklearn-ckpt-2"   # -1: untagged file names (still loadable)


def save_sklearn_weights(path: str, weights, rounds: Optional[int] = None) -> None:
    """``weights`` = the reference's flat exchange list ``coefs_ + intercepts_``: L coefficient
    matrices [in, out] then L intercept vectors, float64 (S:26).  Stored as safetensors keys
    ``coefs_.{i}`` / ``intercepts_.{i}``, float64, same shapes (header: the round, if given)."""
    save_file, _ = _st()
    ws = [np.asarray(w, dtype=np.float64) for w in weights]
    L = len(ws) // 2
    if len(ws) != 2 * L or any(ws[i].ndim != 2 or ws[L + i].shape != (ws[i].shape[1],) for i in range(L)):
        raise ValueError("expected coefs_ ([in, out] matrices) followed by intercepts_ ([out] vectors)")
    t = {f"coefs_.{i}": np.ascontiguousarray(ws[i]) for i in range(L)}
    t.update({f"intercepts_.{i}": np.ascontiguousarray(ws[L + i]) for i in range(L)})
    save_file(t, path, metadata=None if rounds is None else {"round": str(int(rounds))})


def load_sklearn_weights(path: str, expect_round: Optional[int] = None):
    """Inverse of :func:`save_sklearn_weights`: the ``coefs_ + intercepts_`` list, float64."""
    _, load_file = _st()
    _check_round(path, expect_round)
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
    """[S] round checkpoint (collective): every rank writes its local model
    ``client{r}.r<R>.safetensors``, rank 0 ``global.r<R>.safetensors``; after a barrier rank 0
    publishes ``meta.json`` (rounds done, the set's file names, history, run settings), and only
    after a second barrier are older rounds' files pruned.  A crash at any point leaves meta.json
    naming one complete set, and every file's header carries its round, checked on load."""
    os.makedirs(path, exist_ok=True)
    R = int(round_done)
    multi = comm is not None and getattr(comm, "size", 1) > 1
    cname = f"client{rank}.safetensors"
    _atomic(os.path.join(path, tagged(cname, R)), lambda tmp: save_sklearn_weights(tmp, local_weights, R))
    if rank == 0 and global_weights is not None:
        _atomic(os.path.join(path, tagged("global.safetensors", R)),
                lambda tmp: save_sklearn_weights(tmp, global_weights, R))
    if multi:
        comm.Barrier()   # every client file of this round is in place
    if rank == 0:
        files = {"client": tagged("client{rank}.safetensors", R),
                 "global": tagged("global.safetensors", R) if global_weights is not None else None}
        _publish_meta(path, dict(meta, format=SK_FORMAT, rounds=R, files=files))
    if multi:
        comm.Barrier()   # meta.json names round R: older sets may go
    _prune(path, cname, R)
    if rank == 0:
        _prune(path, "global.safetensors", R)


def load_sklearn_run(path: str, rank: int) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    fmt = meta.get("format")
    if fmt not in (SK_FORMAT, "fedmi-sklearn-ckpt-1"):
        raise ValueError(f"{path}: unsupported checkpoint format {fmt!r}")
    R = int(meta["rounds"]) if fmt == SK_FORMAT else None
    files = meta.get("files", {"client": "client{rank}.safetensors", "global": "global.safetensors"})
    out = {"meta": meta,
           "local": load_sklearn_weights(os.path.join(path, files["client"].format(rank=rank)), expect_round=R)}
    gp = os.path.join(path, files["global"]) if files.get("global") else None
    out["global"] = load_sklearn_weights(gp, expect_round=R) if gp and os.path.isfile(gp) else None
    return out
