"""Collective watchdog (the reference has no timeouts).

A daemon thread holds a deadline while a chunk of rounds (kernels + all-reduces) is in
flight.  If the chunk does not complete in time -- a peer died or hung inside a
collective, so this rank is blocked in ``hipStreamSynchronize`` / the all-reduce -- the
watchdog reports which operation stalled and calls ``on_timeout`` (``Comm.Abort``:
``ncclCommAbort`` then a non-zero exit, so the launcher tears the job down) instead of
hanging forever.
"""
from __future__ import annotations

import sys
import threading
import time
from contextlib import contextmanager
from typing import Callable, Optional


class Watchdog:
    def __init__(self, timeout_s: float, on_timeout: Callable[[], None], rank: int = 0):
        self.timeout_s = float(timeout_s)
        self.on_timeout = on_timeout
        self.rank = rank
        self._cv = threading.Condition()
        self._deadline: Optional[float] = None
        self._what = ""
        self._closed = False
        self.fired = False
        self._thread = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._loop, name="fedmi-watchdog", daemon=True)
            self._thread.start()

    def _loop(self) -> None:
        with self._cv:
            while not self._closed:
                if self._deadline is None:
                    self._cv.wait()
                    continue
                left = self._deadline - time.monotonic()
                if left > 0:
                    self._cv.wait(timeout=left)
                    continue
                self.fired = True
                what = self._what
                self._deadline = None
                break
        if self.fired:
            print(f"[watchdog] rank {self.rank}: '{what}' did not complete within {self.timeout_s:.1f}s "
                  f"(peer failure or hang); aborting", file=sys.stderr, flush=True)
            self.on_timeout()

    @contextmanager
    def guard(self, what: str):
        if self._thread is None:
            yield
            return
        with self._cv:
            self._deadline = time.monotonic() + self.timeout_s
            self._what = what
            self._cv.notify()
        try:
            yield
        finally:
            with self._cv:
                self._deadline = None
                self._cv.notify()

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify()
