"""Fault injection for the abort path.

The reference's only failure handling is ``try/except Exception -> comm.Abort()`` around
the round loop (``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:129, 203-205``);
[S]/[H] have none, and an exception on one rank leaves the others blocked in a collective.
``--fault-inject RANK:ROUND[:KIND]`` makes client RANK fail when it reaches round ROUND:

* ``raise`` -- raise inside the round loop (exercises the except -> Abort path, which
  aborts the RCCL communicator and exits non-zero; the launcher tears down the peers);
* ``exit``  -- hard process death without cleanup (a crashed client: peers must be torn
  down by the launcher / their watchdog, not by a cooperative abort);
* ``hang``  -- stop making progress (a wedged client: the peers' collective watchdog
  fires; the hung rank's own watchdog fires too).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Optional

KINDS = ("raise", "exit", "hang")


class InjectedFault(RuntimeError):
    pass


@dataclass(frozen=True)
class FaultSpec:
    rank: int
    round: int
    kind: str = "raise"

    def applies(self, rank: int) -> bool:
        return rank == self.rank

    def trigger(self, rank: int, rnd: int) -> None:
        msg = f"injected fault ({self.kind}) on rank {rank} at round {rnd}"
        print(msg, flush=True)
        if self.kind == "raise":
            raise InjectedFault(msg)
        if self.kind == "exit":
            os._exit(17)
        while True:  # hang
            time.sleep(3600)


def parse_fault(spec: Optional[str]) -> Optional[FaultSpec]:
    if not spec:
        return None
    parts = spec.split(":")
    if len(parts) not in (2, 3):
        raise ValueError(f"--fault-inject expects RANK:ROUND[:KIND], got {spec!r}")
    kind = parts[2] if len(parts) == 3 else "raise"
    if kind not in KINDS:
        raise ValueError(f"fault kind must be one of {KINDS}, got {kind!r}")
    return FaultSpec(int(parts[0]), int(parts[1]), kind)
