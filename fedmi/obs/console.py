"""Reference-format console output and JSONL metric streams.

The reference prints, per round, ``Round r:`` then every rank's local metrics in rank
order (forced by 2*k barriers, C:151-162), then ``Global Metrics`` on rank 0 (C:172-179)
and the early-stop messages (C:135, C:188).  Users parse those lines, so the format is
kept byte-for-byte; but here rank 0 prints *all* ranks' lines from the device-side
metric history (the all-reduced per-rank confusion matrices), so printing costs no
collectives and no barriers.
"""
from __future__ import annotations

import json
import time
from typing import IO, Optional

import numpy as np

from ..fl.metrics import METRIC_NAMES


def _fmt(v) -> str:
    return (f"[accuracy: {v[0]:.4f}, precision: {v[1]:.4f}, "
            f"recall: {v[2]:.4f}, f1: {v[3]:.4f}]")


def format_round(r: int, per_rank: np.ndarray, glob: np.ndarray) -> str:
    lines = [f"\nRound {r + 1}:\n"]
    for k in range(per_rank.shape[0]):
        lines.append(f"  RANK {k} - Local Metrics (Round {r + 1}): {_fmt(per_rank[k])}")
    lines.append(f"  Global Metrics (Round {r + 1}): {_fmt(glob)}")
    return "\n".join(lines)


def print_history(hist: dict, patience: int, start: int = 0, out: Optional[IO] = None,
                  print_fn=print) -> int:
    """Print rounds [start, rounds_run) of an engine history in the reference format;
    returns the next round to print."""
    n = hist["rounds_run"]
    for r in range(start, n):
        print_fn(format_round(r, hist["per_rank"][r], hist["global"][r]), flush=True)
        if hist.get("stop_trigger", -1) == r:
            print_fn(f"Early stopping triggered: No significant change in metrics for {patience} rounds.",
                     flush=True)
    if hist.get("stop_round", -1) >= 0 and n == hist["stop_round"] and start <= n:
        print_fn(f"Training stopped early at round {hist['stop_round']}.", flush=True)
    return n


class JsonlWriter:
    """One JSON object per line (round metrics, timings, bench results)."""

    def __init__(self, path: Optional[str]):
        self.f = open(path, "a") if path else None

    def write(self, **rec) -> None:
        if self.f is None:
            return
        rec.setdefault("ts", time.time())
        self.f.write(json.dumps(rec, default=_default) + "\n")
        self.f.flush()

    def history(self, hist: dict, **extra) -> None:
        for r in range(hist["rounds_run"]):
            self.write(round=r + 1, **{k: float(hist["global"][r][i]) for i, k in enumerate(METRIC_NAMES)},
                       per_rank=hist["per_rank"][r].tolist(), loss=float(hist["loss"][r]), **extra)

    def close(self) -> None:
        if self.f is not None:
            self.f.close()
            self.f = None


def _default(o):
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, (np.floating, np.integer)):
        return o.item()
    raise TypeError(type(o))
