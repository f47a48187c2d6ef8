"""End-of-run replica check: every rank must hold the same global model.

FedAvg's contract (reference ``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:101-120``:
root averages, ``bcast``, every rank ``set_weights``) is that after a round all clients hold
bit-identical global weights.  fedmi's data planes keep that contract by construction
(rank-order sums in the one-shot xGMI kernels; RCCL's all-reduce hands every rank the same
reduced chunks), but a cross-GPU visibility bug -- a stale cache line on one xGMI pull -- would
silently break it and a benchmark would report numbers of a run that was not FedAvg.

:func:`check_replicas` hashes each rank's global image on the host and all-gathers the
digests over the control plane (gloo): one tiny message at the END of a run, never inside
the timed region.
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Union

import numpy as np

ArrayLike = Union[np.ndarray, "torch.Tensor"]  # noqa: F821


def digest(arrays: Iterable[ArrayLike]) -> str:
    """sha256 (16 hex) over the raw bytes of the arrays, in order (dtype and shape included)."""
    h = hashlib.sha256()
    for a in arrays:
        if hasattr(a, "detach"):  # torch tensor (device or host)
            a = a.detach()
            if a.dtype.is_floating_point and a.dtype.itemsize == 2:
                a = a.view(dtype=__import__("torch").int16)
            a = a.cpu().numpy()
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()[:16]


def gather_digests(comm, arrays: Iterable[ArrayLike]) -> List[str]:
    d = digest(arrays)
    if comm is None or comm.size == 1:
        return [d]
    return comm.allgather(d)


def check_replicas(comm, arrays: Iterable[ArrayLike], what: str = "global model", strict: bool = True) -> bool:
    """Collective.  ``True`` if every rank's ``arrays`` hash equal.  With ``strict`` a
    mismatch raises on every rank (all ranks see the same digest list, so they agree)."""
    ds = gather_digests(comm, arrays)
    ok = all(d == ds[0] for d in ds)
    if not ok and strict:
        raise RuntimeError(f"replica check failed: ranks hold different {what}s after FedAvg "
                           f"(per-rank sha256/16: {ds}) -- the data plane lost or reordered an update")
    return ok
