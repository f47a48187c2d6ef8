"""Checkpoint / resume in the reference's weight-exchange layout.

The reference persists nothing; its de-facto checkpoint layout is the in-memory exchange
format: the ``named_parameters()`` dict ``model.{2i}.weight`` [out, in] /
``model.{2i}.bias`` fp32 ([C], C:93-94) and, for sklearn, ``coefs_ + intercepts_``
([in, out], float64; S:26).  A fedmi checkpoint is a directory with

* ``weights.safetensors`` -- the global model under the reference key names (loadable into
  a plain ``torch.nn`` model of the reference with ``load_state_dict``),
* ``optim.safetensors``   -- flat Adam ``exp_avg`` / ``exp_avg_sq`` (these persist across
  rounds in the reference, Q6) and the local weights,
* ``meta.json``           -- dims, rounds done, engine config, early-stop state, history.

Only safetensors / JSON: nothing in a checkpoint can execute code on load.
"""
from __future__ import annotations

import json
import os
from typing import Dict

import numpy as np

from ..models.mlp import dict_to_flat, flat_to_dict


def _st():
    from safetensors.numpy import load_file, save_file
    return save_file, load_file


def save_weights(path: str, weights: Dict[str, np.ndarray]) -> None:
    save_file, _ = _st()
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()}, path)


def load_weights(path: str) -> Dict[str, np.ndarray]:
    _, load_file = _st()
    return dict(load_file(path))


def save_checkpoint(path: str, trainer) -> None:
    eng = trainer.engine if hasattr(trainer, "engine") else trainer
    os.makedirs(path, exist_ok=True)
    sd = eng.state_dict()
    save_weights(os.path.join(path, "weights.safetensors"), flat_to_dict(sd["params"], eng.dims))
    save_file, _ = _st()
    optim = {}
    if "exp_avg" in sd:
        optim["exp_avg"] = np.asarray(sd["exp_avg"], np.float32)
        optim["exp_avg_sq"] = np.asarray(sd["exp_avg_sq"], np.float32)
        optim["local"] = np.asarray(sd["local"], np.float32)
        optim["device_state"] = np.asarray(sd["state"], np.uint8)
    if optim:
        save_file(optim, os.path.join(path, "optim.safetensors"))
    hist = sd.get("history", {})
    meta = {
        "format": "fedmi-ckpt-1",
        "dims": list(eng.dims),
        "rounds": int(sd.get("rounds", 0)),
        "config": eng.cfg.to_dict(),
        "world": eng.world,
        "rank": eng.rank,
        "history": {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in hist.items()},
    }
    if "stopper" in sd:
        meta["stopper"] = sd["stopper"]
    with open(os.path.join(path, "meta.json"), "w") as f:
        json.dump(meta, f)


def load_checkpoint(path: str) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    w = load_weights(os.path.join(path, "weights.safetensors"))
    out = {"meta": meta, "weights": w, "flat": dict_to_flat(w, meta["dims"])}
    op = os.path.join(path, "optim.safetensors")
    if os.path.isfile(op):
        _, load_file = _st()
        out["optim"] = dict(load_file(op))
    return out
