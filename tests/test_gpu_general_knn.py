"""Step 5 beyond the bf16-exact range (MI355X only), and the reference's own
hot-path unit tests re-expressed against grid_amd.

* test/test_neighbors.py:44-75 (find_neighbors_sklearn: nearest pair, self
  excluded, k capped at N-1, squared distance 25.0) and
  test/test_normalize.py:87-111 (normalize_matrix shape / ratio dict,
  select_high_variance_regions) run on the GPU path with the reference's
  inputs and assertions.
* Exact integer hundredths of any magnitude (zmax > 2.56): grid_knn_dist_i32
  vs the oracle's exact distances, bit for bit.
* General fp64 values (e.g. zmax = 2.005 clips): grid_knn_dist_f64 vs the
  oracle's sequential fp64 restatement (oracle.steps.knn_direct_f64), bit for
  bit on the distances, identical neighbour order.
"""
import numpy as np
import pytest

from oracle import steps

pytestmark = pytest.mark.gpu


# ---- the reference's test/test_neighbors.py:44-75, against grid_amd ----
def test_ref_find_neighbors_sklearn_basic():
    from grid_amd.utils.find_neighbors import find_neighbors_sklearn
    data = np.array([[1.0, 0.0], [1.1, 0.1], [5.0, 5.0]])
    result = find_neighbors_sklearn(data, ["S1", "S2", "S3"], n_neighbors=2)
    assert set(result.keys()) == {"S1", "S2", "S3"}
    assert "S2" in [nbr for nbr, _ in result["S1"]]


def test_ref_find_neighbors_sklearn_excludes_self():
    from grid_amd.utils.find_neighbors import find_neighbors_sklearn
    data = np.array([[1.0, 0.0], [2.0, 0.0], [3.0, 0.0]])
    result = find_neighbors_sklearn(data, ["A", "B", "C"], n_neighbors=2)
    for ind, nbrs in result.items():
        assert ind not in [n for n, _ in nbrs]


def test_ref_find_neighbors_sklearn_fewer_than_requested():
    from grid_amd.utils.find_neighbors import find_neighbors_sklearn
    result = find_neighbors_sklearn(np.array([[1.0], [2.0]]), ["A", "B"], n_neighbors=10)
    assert len(result["A"]) == 1


def test_ref_find_neighbors_distances_are_squared():
    from grid_amd.utils.find_neighbors import find_neighbors_sklearn
    result = find_neighbors_sklearn(np.array([[0.0, 0.0], [3.0, 4.0]]), ["A", "B"], n_neighbors=1)
    _, sq_dist = result["A"][0]
    assert sq_dist == pytest.approx(25.0, rel=1e-5)


# ---- the reference's test/test_normalize.py:87-111, against grid_amd ----
def test_ref_normalize_matrix_shape():
    from grid_amd.utils.normalize_mosdepth import normalize_matrix
    mat = np.array([[30.0, 40.0, 35.0], [20.0, 25.0, 22.0], [35.0, 45.0, 40.0]])
    norm, ratios, col_means, col_vars = normalize_matrix(mat)
    assert norm.shape == mat.shape


def test_ref_normalize_matrix_returns_variance_ratios():
    from grid_amd.utils.normalize_mosdepth import normalize_matrix
    mat = np.array([[30.0, 40.0], [20.0, 60.0], [40.0, 20.0]])
    _, ratios, _, _ = normalize_matrix(mat)
    assert isinstance(ratios, dict)
    assert len(ratios) == 2


def test_ref_select_high_variance_regions():
    from grid_amd.utils.normalize_mosdepth import select_high_variance_regions
    selected = select_high_variance_regions({0: 1.0, 1: 5.0, 2: 10.0, 3: 2.0}, top_frac=0.5)
    assert 2 in selected
    assert select_high_variance_regions({}) == []


# ---- general values ----
def _check_int(res, q, k, ids):
    exp = steps.knn_exact(q, k)
    for i, sid in enumerate(ids):
        assert [a for a, _ in res[sid]] == [ids[j] for j, _ in exp[i]], sid
        assert [b for _, b in res[sid]] == [s / 10000.0 for _, s in exp[i]], sid


@pytest.mark.parametrize("n,r,qmax,k,seed", [(70, 300, 2000, 7, 1), (300, 129, 257, 12, 2),
                                             (40, 3000, 50000, 45, 3), (5, 1, 300, 10, 4)])
def test_knn_exact_large_hundredths(n, r, qmax, k, seed):
    """|z| > 2.56: exact int64 direct-difference distances (grid_knn_dist_i32)."""
    from grid_amd.utils.find_neighbors import find_neighbors_sklearn
    rng = np.random.default_rng(seed)
    q = rng.integers(-qmax, qmax + 1, size=(n, r))
    q[0, 0] = qmax
    ids = [f"X{i}" for i in range(n)]
    _check_int(find_neighbors_sklearn(q / 100.0, ids, n_neighbors=k), q, k, ids)


@pytest.mark.parametrize("n,r,k,seed", [(90, 200, 9, 1), (257, 70, 40, 2), (3, 5, 10, 3)])
def test_knn_general_fp64(n, r, k, seed):
    """Values that are not hundredths: the fixed-order fp64 path, bit for bit
    against its restatement."""
    from grid_amd import engine
    from grid_amd.device import get_device
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, r)) * 1.7
    idx, d2, cnt = engine.knn_values(get_device(), x, k)
    exp = steps.knn_direct_f64(x, k)
    for i in range(n):
        assert cnt[i] == len(exp[i])
        assert idx[i, : cnt[i]].tolist() == [j for j, _ in exp[i]], i
        assert d2[i, : cnt[i]].tolist() == [s for _, s in exp[i]], i


@pytest.mark.parametrize("zmax", [3.0, 2.005, 0.5])
def test_knn_from_zq_any_zmax(zmax):
    """find_neighbors' clip/NaN/column filter on the int32 step-4 hundredths for
    zmax values off the bf16 fast path (3.0: exact int; 2.005: fp64) and on it
    (0.5), against the reference's float arithmetic (np.clip on q/100)."""
    from grid_amd import _abi, engine
    from grid_amd.device import get_device
    rng = np.random.default_rng(int(zmax * 1000))
    n, m = 120, 500
    zq = rng.integers(-450, 451, size=(n, m)).astype(np.int32)
    zq[rng.random((n, m)) < 0.02] = _abi.MISSING
    cols = np.sort(rng.choice(m, 400, replace=False)).astype(np.int32)
    idx, d2, cnt = engine.knn_from_zq(get_device(), zq, cols, 8, zmax)
    data = np.where(zq == _abi.MISSING, np.nan, zq / 100.0)[:, cols]
    data = np.nan_to_num(np.clip(data, -zmax, zmax), nan=0.0)            # find_neighbors.py:57-58
    qv = np.rint(data * 100)
    if np.array_equal(qv / 100.0, data):
        exp = [[(j, s / 10000.0) for j, s in row] for row in steps.knn_exact(qv.astype(np.int64), 8)]
    else:
        exp = steps.knn_direct_f64(data, 8)
    for i in range(n):
        assert idx[i, : cnt[i]].tolist() == [j for j, _ in exp[i]], i
        assert d2[i, : cnt[i]].tolist() == [s for _, s in exp[i]], i
