"""R producer: the sparse random matrix of sklearn's ``SparseRandomProjection``.

The reference builds R on the Spark driver with
``SparseRandomProjection(n_components=p, random_state=123).fit(dummy_X)``
(``code/clustermode/randomProjection.py:93-96``, ``code/localmode/randomProjection.py:114-121``)
and then ships ``srp.components_.T.astype(np.float32)`` (``clustermode/randomProjection.py:101``).
The arithmetic lives in scikit-learn (not vendored in the reference):

* ``sklearn/random_projection.py:209-304`` ``_sparse_random_matrix``: per component
  ``n_nonzero_i = rng.binomial(n_features, density)``, indices from
  ``sample_without_replacement``, then ``data = rng.binomial(1, .5, nnz) * 2 - 1`` and the scale
  ``sqrt(1 / density) / sqrt(n_components)``.
* ``sklearn/utils/_random.pyx:44-106`` tracking selection (rejection with a set, one
  ``rng.randint(n_population)`` per draw), ``:225-268`` the method dispatch (``rng.permutation``
  when 0.01 < ratio < 0.99, reservoir sampling when ratio >= 0.2 otherwise).
* ``sklearn/random_projection.py:367-431`` ``fit`` casts with ``.astype(X.dtype)``.

This module restates that stream with vectorised numpy calls that consume the legacy
``RandomState`` (MT19937) stream exactly as the scalar calls do, so the matrix is bit-identical
to sklearn's (pinned by ``tests/test_srp_matrix.py`` against sklearn-made fixtures and the
full-size KDD2012 digests of SURVEY.md §8(c)). It takes seconds instead of the ~45 s of the
per-draw Python loop.
"""
from __future__ import annotations

import hashlib
import math

import numpy as np
import scipy.sparse as sp

__all__ = [
    "auto_density",
    "check_density",
    "sample_without_replacement",
    "sparse_random_matrix",
    "gaussian_random_matrix",
    "johnson_lindenstrauss_min_dim",
    "projection_operand",
    "csr_digest",
]


def auto_density(n_features: int) -> float:
    """``density='auto'`` = 1/sqrt(n_features) (sklearn/random_projection.py ``_check_density``)."""
    return 1.0 / np.sqrt(n_features)


def check_density(density, n_features: int) -> float:
    """Mirror of sklearn ``_check_density``: 'auto' -> 1/sqrt(m); must lie in (0, 1]."""
    if isinstance(density, str) and density == "auto":
        density = auto_density(n_features)
    if density <= 0 or density > 1:
        raise ValueError("Expected density in range ]0, 1], got: %r" % density)
    return density


def johnson_lindenstrauss_min_dim(n_samples, *, eps=0.1):
    """JL lower bound used by ``code/localmode/randomProjection.py:112`` (sklearn
    ``random_projection.py:63-146``): ``4 log(n) / (eps^2/2 - eps^3/3)`` truncated to int."""
    eps = np.asarray(eps)
    n_samples = np.asarray(n_samples)
    if np.any(eps <= 0.0) or np.any(eps >= 1):
        raise ValueError("The JL bound is defined for eps in ]0, 1[, got %r" % eps)
    if np.any(n_samples <= 0):
        raise ValueError("The JL bound is defined for n_samples greater than zero, got %r" % n_samples)
    denominator = (eps**2 / 2) - (eps**3 / 3)
    return (4 * np.log(n_samples) / denominator).astype(np.int64)


def _tracking_selection(rng: np.random.RandomState, n_population: int, n_samples: int) -> np.ndarray:
    """Vectorised restatement of ``_sample_without_replacement_with_tracking_selection``
    (sklearn/utils/_random.pyx:92-104): draw ``randint(n_population)`` until ``n_samples``
    distinct values were accepted, in acceptance order.

    A vector draw of size k consumes the MT19937 stream exactly like k scalar draws, and the
    scalar loop needs at least ``n_samples - accepted`` more draws at any point, so drawing
    exactly that many and accepting first occurrences reproduces its output and its final state.
    """
    out = np.empty(n_samples, dtype=np.int64)
    filled = 0
    seen = None
    while filled < n_samples:
        need = n_samples - filled
        draws = rng.randint(n_population, size=need)
        _, first = np.unique(draws, return_index=True)
        first.sort()
        cand = draws[first]
        if seen is not None:
            cand = cand[~np.isin(cand, out[:filled], assume_unique=True)]
        out[filled:filled + cand.size] = cand
        filled += cand.size
        seen = True
    return out


def _reservoir_sampling(rng: np.random.RandomState, n_population: int, n_samples: int) -> np.ndarray:
    """Vectorised ``_sample_without_replacement_with_reservoir_sampling`` (sklearn/utils/_random.pyx):
    ``out[i] = i`` then for i in [n_samples, n_population): ``j = randint(0, i+1)``; if j < n_samples:
    ``out[j] = i``. The later i wins for a repeated j."""
    out = np.arange(n_samples, dtype=np.int64)
    if n_population > n_samples:
        i = np.arange(n_samples, n_population, dtype=np.int64)
        j = rng.randint(0, i + 1)
        keep = j < n_samples
        i, j = i[keep], j[keep]
        # last write wins: take the largest i per j
        order = np.lexsort((i, j))
        j, i = j[order], i[order]
        last = np.ones(j.size, dtype=bool)
        last[:-1] = j[1:] != j[:-1]
        out[j[last]] = i[last]
    return out


def sample_without_replacement(n_population: int, n_samples: int, rng: np.random.RandomState) -> np.ndarray:
    """Method ``'auto'`` dispatch of sklearn/utils/_random.pyx:225-256."""
    if n_population < 0:
        raise ValueError("n_population should be greater than 0, got %s." % n_population)
    if n_samples > n_population:
        raise ValueError(
            "n_population should be greater or equal than n_samples, got n_samples > n_population (%s > %s)"
            % (n_samples, n_population))
    ratio = n_samples / n_population if n_population != 0 else 1.0
    if 0.01 < ratio < 0.99:
        return rng.permutation(n_population)[:n_samples]
    if ratio < 0.2:
        return _tracking_selection(rng, n_population, n_samples)
    return _reservoir_sampling(rng, n_population, n_samples)


def _as_rng(random_state) -> np.random.RandomState:
    if random_state is None or random_state is np.random:
        return np.random.mtrand._rand
    if isinstance(random_state, (int, np.integer)):
        return np.random.RandomState(random_state)
    if isinstance(random_state, np.random.RandomState):
        return random_state
    raise ValueError("%r cannot be used to seed a numpy.random.RandomState instance" % random_state)


def sparse_random_matrix(n_components: int, n_features: int, density="auto", random_state=None):
    """Bit-identical restatement of sklearn ``_sparse_random_matrix`` (random_projection.py:209-304).

    Returns the (n_components, n_features) ``csr_matrix`` with float64 values (unsorted indices
    within a row, like sklearn), or a dense ndarray when density == 1.
    """
    if n_components <= 0:
        raise ValueError("n_components must be strictly positive, got %d" % n_components)
    if n_features <= 0:
        raise ValueError("n_features must be strictly positive, got %d" % n_features)
    density = check_density(density, n_features)
    rng = _as_rng(random_state)
    if density == 1:
        components = rng.binomial(1, 0.5, (n_components, n_features)) * 2 - 1
        return 1 / np.sqrt(n_components) * components
    indices = []
    indptr = np.zeros(n_components + 1, dtype=np.int64)
    for i in range(n_components):
        k = rng.binomial(n_features, density)
        indices.append(sample_without_replacement(n_features, k, rng))
        indptr[i + 1] = indptr[i] + k
    indices = np.concatenate(indices) if indices else np.zeros(0, dtype=np.int64)
    data = rng.binomial(1, 0.5, size=np.size(indices)) * 2 - 1
    components = sp.csr_matrix((data, indices, indptr), shape=(n_components, n_features))
    return np.sqrt(1 / density) / np.sqrt(n_components) * components


def gaussian_random_matrix(n_components: int, n_features: int, random_state=None) -> np.ndarray:
    """sklearn ``_gaussian_random_matrix`` (random_projection.py:169-206): N(0, 1/sqrt(p))."""
    rng = _as_rng(random_state)
    return rng.normal(loc=0.0, scale=1.0 / np.sqrt(n_components), size=(n_components, n_features))


def projection_operand(components, dtype=np.float32) -> sp.csr_matrix:
    """The right operand the recipe multiplies by: ``components_.T.astype(float32)``
    (clustermode/randomProjection.py:101) converted to CSR exactly as scipy's ``_matmul_sparse``
    does (``self.__class__(other)``: CSC -> CSR via csc_tocsr, rows sorted by component)."""
    return sp.csr_matrix(components.T.astype(dtype))


def csr_digest(indptr, indices, data) -> str:
    """SURVEY.md §8(c) digest recipe: sha256(indptr <i8 || indices <i4 || data <f4)."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(indptr, dtype="<i8").tobytes())
    h.update(np.ascontiguousarray(indices, dtype="<i4").tobytes())
    h.update(np.ascontiguousarray(data, dtype="<f4").tobytes())
    return h.hexdigest()


# KDD2012 shape, random_state=123, p=4096 (sklearn 1.7.2, measured in the container).
KDD_M = 54_686_452
KDD_P = 4096
KDD_R_CSR_DIGEST = "51e3282ba4169367e3e8910370d9ef2593370781b90998a522d3f2c3842820c2"
KDD_COMPONENTS_DIGEST = "723ac21a65d078f945cd57aed9bf53de5d2d68be0b6407b02fc02126fc594f46"


# ------------------------------------------------------------------------------------------------
# persistence: replaces the joblib pickle of the fitted estimator
# (code/localmode/randomProjection.py:114-121 load-or-fit `srp_{p}.pkl`,
#  code/clustermode/randomProjection.py:98 `joblib.dump(srp, "/tmp/srp.pkl")`).
# Plain arrays in an .npz (no pickle, loadable with allow_pickle=False) plus the SURVEY digest.

def save_components(path, components, *, random_state=None, density=None) -> str:
    """Write ``components_`` (CSR, n_components x n_features) to ``path`` (.npz). Returns the digest
    of the canonical (sorted) CSR, stored alongside and checked on load."""
    C = sp.csr_matrix(components)
    Cs = C.copy()
    Cs.sort_indices()
    digest = csr_digest(Cs.indptr, Cs.indices, Cs.data)
    meta = np.array([C.shape[0], C.shape[1], -1 if random_state is None else int(random_state)], dtype=np.int64)
    np.savez(path, indptr=C.indptr, indices=C.indices, data=C.data, meta=meta,
             density=np.array([np.nan if density is None else float(density)]),
             digest=np.frombuffer(digest.encode(), dtype=np.uint8))
    return digest


def load_components(path, verify: bool = True) -> sp.csr_matrix:
    """Read a matrix written by ``save_components``; ``verify`` re-checks its digest."""
    with np.load(path, allow_pickle=False) as z:
        n, m = int(z["meta"][0]), int(z["meta"][1])
        C = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, m))
        digest = bytes(z["digest"]).decode()
    if verify:
        Cs = C.copy()
        Cs.sort_indices()
        if csr_digest(Cs.indptr, Cs.indices, Cs.data) != digest:
            raise ValueError(f"{path}: digest mismatch (corrupt or edited projection matrix)")
    return C


def load_or_fit(path, n_components: int, n_features: int, random_state=123, density="auto", dtype=np.float32):
    """localmode's load-or-fit cache (code/localmode/randomProjection.py:114-121) without pickles:
    returns ``components_`` cast to ``dtype`` (the fit's ``astype(X.dtype)``)."""
    import os

    if os.path.exists(path):
        C = load_components(path)
        if C.shape != (n_components, n_features):
            raise ValueError(f"{path}: cached shape {C.shape} != {(n_components, n_features)}")
        return C.astype(dtype)
    C = sparse_random_matrix(n_components, n_features, density=density, random_state=random_state).astype(dtype)
    save_components(path, C, random_state=random_state if isinstance(random_state, (int, np.integer)) else None,
                    density=check_density(density, n_features))
    return C
