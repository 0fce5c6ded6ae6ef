"""R producer: bit-identical to sklearn's SparseRandomProjection (every sampling branch) and to
the full-size KDD2012 digests recorded in SURVEY.md §8(c)."""
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr, same_bits
from randomprojection_amd import srp_matrix as sm

warnings.filterwarnings("ignore")


def _sk(m, p, density="auto", dtype=np.float64):
    from sklearn.random_projection import SparseRandomProjection
    return SparseRandomProjection(n_components=p, density=density, random_state=123).fit(
        sp.csr_matrix((10, m), dtype=dtype)).components_


def test_matches_committed_sklearn_fixtures(golden):
    for name, (m, p, dt) in {"comp1": (100_000, 256, np.float32), "comp2": (5000, 64, np.float64)}.items():
        ref = golden_csr(golden, name)
        ours = sm.sparse_random_matrix(p, m, random_state=123).astype(dt)
        assert np.array_equal(ours.indptr, ref.indptr)
        assert np.array_equal(ours.indices, ref.indices)      # same (unsorted) storage order
        assert same_bits(ours.data, ref.data)


@pytest.mark.parametrize("m,p,density", [
    (100_000, 64, "auto"),     # tracking selection
    (5000, 32, "auto"),        # rng.permutation branch (0.01 < 1/sqrt(m) < 0.99)
    (300, 20, 0.995),          # reservoir sampling branch
    (2000, 30, 0.3),           # permutation with explicit density
    (1000, 16, 0.001),         # tiny density, empty rows possible
    (50, 8, 1.0),              # dense branch
])
def test_matches_live_sklearn(m, p, density):
    ref = _sk(m, p, density)
    ours = sm.sparse_random_matrix(p, m, density=density, random_state=123)
    if sp.issparse(ref):
        assert np.array_equal(ours.indptr, ref.indptr) and np.array_equal(ours.indices, ref.indices)
        assert same_bits(ours.data, ref.data)
    else:
        assert same_bits(np.asarray(ours), np.asarray(ref))


def test_randomstate_instance_and_stream_position():
    rs1, rs2 = np.random.RandomState(7), np.random.RandomState(7)
    from sklearn.random_projection import _sparse_random_matrix
    a = sm.sparse_random_matrix(16, 20_000, random_state=rs1)
    b = _sparse_random_matrix(16, 20_000, random_state=rs2)
    assert np.array_equal(a.indices, b.indices)
    assert rs1.randint(1 << 30) == rs2.randint(1 << 30)   # identical stream consumption


def test_jl_min_dim():
    from sklearn.random_projection import johnson_lindenstrauss_min_dim as sk
    for n, eps in [(119_705_032, 0.2), (1_077_345_288, 0.2), (1000, 0.1)]:
        assert sm.johnson_lindenstrauss_min_dim(n, eps=eps) == sk(n, eps=eps)
    assert sm.johnson_lindenstrauss_min_dim(119_705_032, eps=0.2) == 4292   # localmode:112


def test_bad_density():
    with pytest.raises(ValueError):
        sm.sparse_random_matrix(4, 100, density=0.0)


@pytest.mark.slow
def test_full_kdd_digest():
    """54,686,452 x 4096, random_state=123: both digests of SURVEY.md §8(c)."""
    C = sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123)
    assert C.nnz == 30_302_336
    c32 = C.astype(np.float32)
    R = sm.projection_operand(C)
    assert sm.csr_digest(R.indptr, R.indices, R.data) == sm.KDD_R_CSR_DIGEST
    c32.sort_indices()
    assert sm.csr_digest(c32.indptr, c32.indices, c32.data) == sm.KDD_COMPONENTS_DIGEST


def test_npz_persistence_roundtrip(tmp_path):
    path = tmp_path / "srp_256.npz"
    C = sm.load_or_fit(str(path), 256, 100_000)          # fits and saves
    assert path.exists()
    C2 = sm.load_or_fit(str(path), 256, 100_000)         # loads (no pickle) and verifies the digest
    assert np.array_equal(C.indices, C2.indices) and same_bits(C.data, C2.data)
    ref = _sk(100_000, 256, dtype=np.float32)
    assert np.array_equal(C2.indices, ref.indices) and same_bits(C2.data, ref.data)
    z = dict(np.load(path, allow_pickle=False))
    z["data"] = z["data"].copy()
    z["data"][0] *= -1
    np.savez(path, **z)
    with pytest.raises(ValueError, match="digest"):
        sm.load_components(str(path))
    sm.save_components(str(path), C)
    with pytest.raises(ValueError, match="shape"):
        sm.load_or_fit(str(path), 128, 100_000)


def test_gaussian_matrix_matches_sklearn():
    from sklearn.random_projection import GaussianRandomProjection
    X = np.zeros((5, 3000), dtype=np.float32)
    ref = GaussianRandomProjection(n_components=64, random_state=123).fit(X).components_
    ours = sm.gaussian_random_matrix(64, 3000, random_state=123).astype(np.float32)
    assert same_bits(ours, ref)
