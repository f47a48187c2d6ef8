"""Host-side tabular data pipeline (CSV -> label-encode -> scale -> split).

Re-creates the preprocessing every reference entrypoint runs before training
(reference ``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:216-246``,
``FL_SkLearn_MLPClassifier_Limitation.py:163-197``, ``hyperparameters_tuning.py:143-177``):

* every ``object`` column is label-encoded with *sorted* class codes
  (sklearn ``LabelEncoder`` semantics, C:222-228),
* features are standardised over the *full* table before the split
  (``StandardScaler()`` in [C] C:235, ``with_mean=False`` in [S]/[H] S:184),
* ``train_test_split(test_size=0.2, random_state=42)`` (C:239).

Everything here is numpy: the table is 10 000 rows and is loaded exactly once per
process.  Unlike the reference there is no rank-0 split + pickle broadcast
(C:243-246): the split is deterministic, so every rank derives it locally and
keeps only its own shard (first row).
"""
from __future__ import annotations

import csv
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

DEFAULT_DATASET = "balanced_income_data.csv"
DEFAULT_LABEL = "income"


def find_dataset(name: str = DEFAULT_DATASET) -> str:
    """Locate the dataset: explicit path, CWD, the repo's ``data/`` dir, then the
    read-only reference checkout."""
    candidates = [name, os.path.join(os.getcwd(), name)]
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(os.path.dirname(here))
    candidates.append(os.path.join(repo, "data", os.path.basename(name)))
    candidates.append(os.path.join("/root/reference", os.path.basename(name)))
    for c in candidates:
        if os.path.isfile(c):
            return c
    raise FileNotFoundError(f"dataset {name!r} not found (tried {candidates})")


@dataclass
class Table:
    columns: List[str]
    data: Dict[str, np.ndarray]
    encoders: Dict[str, np.ndarray] = field(default_factory=dict)  # column -> sorted classes

    def __len__(self) -> int:
        return len(next(iter(self.data.values()))) if self.data else 0


def _parse_column(values: List[str]) -> np.ndarray:
    """pandas-like dtype inference: int64 if every cell parses as int, else float64,
    else object (kept as a numpy array of str)."""
    try:
        return np.array([int(v) for v in values], dtype=np.int64)
    except ValueError:
        pass
    try:
        return np.array([float(v) for v in values], dtype=np.float64)
    except ValueError:
        return np.array(values, dtype=object)


def read_csv(path: str) -> Table:
    with open(path, newline="") as f:
        reader = csv.reader(f)
        header = next(reader)
        rows = [r for r in reader if r]
    cols = list(zip(*rows)) if rows else [[] for _ in header]
    data = {h: _parse_column(list(c)) for h, c in zip(header, cols)}
    return Table(columns=list(header), data=data)


def encode_categorical_features(table: Table) -> Table:
    """LabelEncoder per object column: codes are indices into the sorted unique
    classes (reference C:222-228)."""
    for c in table.columns:
        col = table.data[c]
        if col.dtype == object:
            classes, codes = np.unique(col.astype(str), return_inverse=True)
            table.data[c] = codes.astype(np.int64)
            table.encoders[c] = classes
    return table


class StandardScaler:
    """Population-std standardiser (sklearn semantics: ddof=0, zero std -> 1)."""

    def __init__(self, with_mean: bool = True, with_std: bool = True):
        self.with_mean = with_mean
        self.with_std = with_std
        self.mean_: Optional[np.ndarray] = None
        self.scale_: Optional[np.ndarray] = None

    def fit(self, X: np.ndarray) -> "StandardScaler":
        X = np.asarray(X, dtype=np.float64)
        self.mean_ = X.mean(axis=0)
        var = X.var(axis=0)
        scale = np.sqrt(var)
        scale[scale == 0.0] = 1.0
        self.scale_ = scale
        return self

    def transform(self, X: np.ndarray) -> np.ndarray:
        X = np.asarray(X, dtype=np.float64)
        out = X - self.mean_ if self.with_mean else X.copy()
        if self.with_std:
            out = out / self.scale_
        return out

    def fit_transform(self, X: np.ndarray) -> np.ndarray:
        return self.fit(X).transform(X)


def train_test_split(X: np.ndarray, y: np.ndarray, test_size: float = 0.2, random_state: int = 42):
    """Bit-exact re-implementation of sklearn's ``train_test_split`` for the
    shuffled, unstratified case (ShuffleSplit: test = perm[:n_test],
    train = perm[n_test:n_test + n_train])."""
    n = len(X)
    n_test = int(math.ceil(test_size * n)) if isinstance(test_size, float) else int(test_size)
    n_train = n - n_test
    perm = np.random.RandomState(random_state).permutation(n)
    test_idx = perm[:n_test]
    train_idx = perm[n_test:n_test + n_train]
    return X[train_idx], X[test_idx], y[train_idx], y[test_idx]


@dataclass
class Dataset:
    X_train: np.ndarray
    y_train: np.ndarray
    X_test: np.ndarray
    y_test: np.ndarray
    feature_names: List[str]
    classes: np.ndarray

    @property
    def n_features(self) -> int:
        return self.X_train.shape[1]

    @property
    def n_classes(self) -> int:
        return int(len(self.classes))


def load_tabular(path: Optional[str] = None, label: str = DEFAULT_LABEL, with_mean: bool = True,
                 test_size: float = 0.2, random_state: int = 42) -> Dataset:
    """Full reference preprocessing pipeline.

    ``with_mean=True`` reproduces [C] (C:235); ``with_mean=False`` reproduces [S]/[H]
    (S:184, H:164).  Raises ``KeyError`` for a missing label column exactly like
    C:219-220.
    """
    path = find_dataset(path or DEFAULT_DATASET)
    table = read_csv(path)
    if label not in table.columns:
        raise KeyError(f"'{label}' not found in dataset columns. Available columns: {table.columns}")
    table = encode_categorical_features(table)
    feats = [c for c in table.columns if c != label]
    X = np.stack([table.data[c].astype(np.float64) for c in feats], axis=1)
    y = table.data[label].astype(np.int64)
    X = StandardScaler(with_mean=with_mean).fit_transform(X)
    X_tr, X_te, y_tr, y_te = train_test_split(X, y, test_size=test_size, random_state=random_state)
    classes = table.encoders.get(label, np.unique(y))
    return Dataset(X_tr, y_tr, X_te, y_te, feats, np.asarray(classes))


def as_float32(X: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(X, dtype=np.float32)


def describe(ds: Dataset) -> str:
    return (f"train {ds.X_train.shape} test {ds.X_test.shape} features={ds.n_features} "
            f"classes={list(ds.classes)}")


__all__ = [
    "DEFAULT_DATASET", "DEFAULT_LABEL", "Dataset", "StandardScaler", "Table", "as_float32",
    "describe", "encode_categorical_features", "find_dataset", "load_tabular", "read_csv",
    "train_test_split",
]


