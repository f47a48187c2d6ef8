"""Early-stopping rule of the [C] round loop.

Reference: ``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:181-192`` --
``np.allclose(avg, prev, atol=tolerance)`` (implicit ``rtol=1e-5``) over the 4-metric
vector; ``prev`` is only replaced on a *significant* change, the patience counter is
reset there and decremented otherwise; reaching 0 sets the stop signal, which takes
effect at the top of the next round (C:132-136), after that round's FedAvg (C:198).

The same rule runs on the device inside the round engine (``fl_finalize_round`` in
``fedmi/ops/csrc/fl_kernels.hip``) so no host round trip or stop-signal broadcast is
needed: every rank evaluates it on identical all-reduced metrics (SURVEY §2.4, C:132).
This host class is the oracle for that kernel and the implementation used on CPU.
"""
from __future__ import annotations

from typing import Optional

import numpy as np


def allclose(a, b, atol: float, rtol: float = 1e-5) -> bool:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return bool(np.all(np.abs(a - b) <= atol + rtol * np.abs(b)))


class EarlyStopper:
    def __init__(self, patience: int = 10, tolerance: float = 1e-4, rtol: float = 1e-5,
                 enabled: bool = True):
        self.patience = int(patience)
        self.tolerance = float(tolerance)
        self.rtol = float(rtol)
        self.enabled = enabled
        self.count = self.patience
        self.prev: Optional[np.ndarray] = None
        self.stopped = False

    def update(self, metric_vec) -> bool:
        """Feed one round's global metric vector; returns True when the stop signal is set."""
        v = np.asarray(metric_vec, dtype=np.float64)
        if not self.enabled:
            return False
        if self.prev is not None and allclose(v, self.prev, self.tolerance, self.rtol):
            self.count -= 1
            if self.count == 0:
                self.stopped = True
        else:
            self.prev = v
            self.count = self.patience
        return self.stopped

    def state_dict(self) -> dict:
        return {"patience": self.patience, "tolerance": self.tolerance, "count": self.count,
                "prev": None if self.prev is None else self.prev.tolist(), "stopped": self.stopped}

    def load_state_dict(self, d: dict) -> None:
        self.patience = int(d["patience"])
        self.tolerance = float(d["tolerance"])
        self.count = int(d["count"])
        self.prev = None if d["prev"] is None else np.asarray(d["prev"], dtype=np.float64)
        self.stopped = bool(d["stopped"])
