"""Client shard assignment.

Four partitioners behind one function, :func:`shard_indices`:

``contiguous``
    [S]/[H] ``_split_data`` (``FL_SkLearn_MLPClassifier_Limitation.py:17-22``): a disjoint,
    contiguous partition with ``chunk = max(1, n // size)`` and the remainder on the last
    rank.
``compat``
    [C] ``_split_data`` (``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:48-61``):
    every rank draws its *own* permutation and slices chunk ``rank`` out of it, so shards
    overlap.  The reference permutation is unseeded; here it is seeded with
    ``seed + rank`` so runs are reproducible while keeping the overlap statistics.
``iid``
    The "correct" mode: one permutation shared by all ranks (same seed), then contiguous
    chunks -> disjoint, exhaustive shards.
``label_skew``
    Non-IID: per-class Dirichlet(alpha) proportions over clients (north-star FedProx
    config).  Deterministic for a given seed, identical on every rank.

All partitioners are deterministic functions of ``(n, labels, rank, size, seed)``, so a
rank never needs to receive another rank's data: there is no broadcast of the training
table (reference C:243-246).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

MODES = ("contiguous", "compat", "iid", "label_skew")


def _chunk(n: int, rank: int, size: int) -> slice:
    chunk = max(1, n // size)
    start = rank * chunk
    end = start + chunk if rank != size - 1 else n
    return slice(min(start, n), min(end, n))


def shard_indices(n: int, rank: int, size: int, mode: str = "iid", seed: int = 0,
                  labels: Optional[np.ndarray] = None, alpha: float = 0.5) -> np.ndarray:
    if not 0 <= rank < size:
        raise ValueError(f"rank {rank} out of range for size {size}")
    if mode == "contiguous":
        return np.arange(n)[_chunk(n, rank, size)]
    if mode == "compat":
        perm = np.random.RandomState(seed + rank).permutation(n)
        return perm[_chunk(n, rank, size)]
    if mode == "iid":
        perm = np.random.RandomState(seed).permutation(n)
        return np.sort(perm[_chunk(n, rank, size)])
    if mode == "label_skew":
        if labels is None:
            raise ValueError("label_skew sharding needs labels")
        return _label_skew(labels, rank, size, seed, alpha)
    raise ValueError(f"unknown shard mode {mode!r}; expected one of {MODES}")


def _label_skew(labels: np.ndarray, rank: int, size: int, seed: int, alpha: float) -> np.ndarray:
    rng = np.random.RandomState(seed)
    labels = np.asarray(labels)
    owners = np.empty(len(labels), dtype=np.int64)
    for c in np.unique(labels):
        idx = np.flatnonzero(labels == c)
        idx = idx[rng.permutation(len(idx))]
        p = rng.dirichlet(np.full(size, alpha))
        cuts = (np.cumsum(p)[:-1] * len(idx)).astype(np.int64)
        for r, part in enumerate(np.split(idx, cuts)):
            owners[part] = r
    # guarantee every client at least one row so collectives never deadlock
    for r in range(size):
        if not np.any(owners == r):
            donor = np.bincount(owners, minlength=size).argmax()
            owners[np.flatnonzero(owners == donor)[0]] = r
    return np.flatnonzero(owners == rank)


def split_data(X: np.ndarray, y: np.ndarray, rank: int, size: int, mode: str = "iid", seed: int = 0,
               alpha: float = 0.5):
    idx = shard_indices(len(X), rank, size, mode=mode, seed=seed, labels=y, alpha=alpha)
    return X[idx], y[idx]


def coverage(n: int, size: int, mode: str, seed: int = 0, labels=None) -> float:
    """Fraction of rows held by at least one client (1.0 for partitions; ~0.66-0.75 for
    the reference's overlapping ``compat`` shards)."""
    seen = np.zeros(n, dtype=bool)
    for r in range(size):
        seen[shard_indices(n, r, size, mode=mode, seed=seed, labels=labels)] = True
    return float(seen.mean())
