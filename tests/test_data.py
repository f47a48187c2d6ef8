"""Data pipeline parity with the reference preprocessing (C:216-246, S:163-197)."""
import numpy as np
import pytest

from fedmi.data.sharding import coverage, shard_indices, split_data
from fedmi.data.synthetic import make_income_like
from fedmi.data.tabular import StandardScaler, load_tabular, train_test_split

sk = pytest.importorskip("sklearn")
pd = pytest.importorskip("pandas")


@pytest.mark.parametrize("with_mean", [True, False])
def test_pipeline_matches_sklearn_pandas(with_mean):
    from sklearn.model_selection import train_test_split as sk_split
    from sklearn.preprocessing import LabelEncoder
    from sklearn.preprocessing import StandardScaler as SkScaler
    from fedmi.data.tabular import find_dataset
    ds = load_tabular(with_mean=with_mean)
    data = pd.read_csv(find_dataset())
    for c in data.select_dtypes(include=["object"]).columns:
        data[c] = LabelEncoder().fit_transform(data[c])
    X = SkScaler(with_mean=with_mean).fit_transform(data.drop("income", axis=1).values)
    y = data["income"].values
    a, b, c, d = sk_split(X, y, test_size=0.2, random_state=42)
    np.testing.assert_allclose(ds.X_train, a, atol=1e-12)
    np.testing.assert_allclose(ds.X_test, b, atol=1e-12)
    assert (ds.y_train == c).all() and (ds.y_test == d).all()
    assert ds.X_train.shape == (8000, 14) and ds.n_classes == 2
    assert list(ds.classes) == ["<=50K", ">50K"]


def test_missing_label_raises_keyerror():
    with pytest.raises(KeyError):
        load_tabular(label="Outcome")


def test_split_bit_exact_small():
    from sklearn.model_selection import train_test_split as sk_split
    X = np.arange(40).reshape(20, 2)
    y = np.arange(20)
    for a, b in zip(train_test_split(X, y, 0.2, 7), sk_split(X, y, test_size=0.2, random_state=7)):
        assert (a == b).all()


def test_scaler_matches_sklearn():
    from sklearn.preprocessing import StandardScaler as SkScaler
    X = np.random.RandomState(0).randn(50, 4) * [1, 10, 0, 3]
    for wm in (True, False):
        np.testing.assert_allclose(StandardScaler(with_mean=wm).fit_transform(X),
                                   SkScaler(with_mean=wm).fit_transform(X), atol=1e-12)


@pytest.mark.parametrize("size", [1, 2, 3, 4, 8])
def test_contiguous_partition(size):
    n = 8000
    parts = [shard_indices(n, r, size, "contiguous") for r in range(size)]
    assert sum(len(p) for p in parts) == n
    assert len(np.unique(np.concatenate(parts))) == n
    chunk = n // size
    assert all(len(p) == chunk for p in parts[:-1])


def test_iid_disjoint_and_compat_overlap():
    n = 8000
    assert coverage(n, 4, "iid") == 1.0
    cov = coverage(n, 4, "compat")
    assert 0.6 < cov < 0.8          # ~69 % at 4 clients
    assert len(shard_indices(n, 1, 2, "compat")) == 4000


def test_label_skew_partition_covers_everything():
    y = np.random.RandomState(0).randint(0, 2, 1000)
    parts = [shard_indices(1000, r, 4, "label_skew", seed=3, labels=y, alpha=0.3) for r in range(4)]
    allp = np.concatenate(parts)
    assert len(allp) == 1000 and len(np.unique(allp)) == 1000
    assert all(len(p) > 0 for p in parts)
    fracs = [y[p].mean() for p in parts]
    assert max(fracs) - min(fracs) > 0.1   # actually skewed


def test_split_data_shapes():
    X = np.zeros((10, 3)); y = np.arange(10)
    Xa, ya = split_data(X, y, 1, 3, mode="contiguous")
    assert (ya == [3, 4, 5]).all()


def test_synthetic_balanced():
    X, y = make_income_like(4000, seed=0)
    assert X.shape == (4000, 14) and X.dtype == np.float32
    assert abs(y.mean() - 0.5) < 0.01
