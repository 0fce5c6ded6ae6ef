"""sklearn-compatible ``SparseRandomProjection`` whose ``transform`` runs on the MI355X.

Drop-in for the estimator the reference fits and ships
(code/clustermode/randomProjection.py:93-101, code/localmode/randomProjection.py:114-127) and for
sklearn's ``transform(X)`` on CSR input (sklearn/random_projection.py:801-824 ->
``safe_sparse_dot(X, components_.T)``, sklearn/utils/extmath.py:153).

* ``fit`` produces the identical ``components_`` (``randomprojection_amd.srp_matrix`` restates
  sklearn's generator bit for bit, vectorised).
* ``transform(X)`` for CSR X returns exactly what sklearn returns: ``X @ components_.T`` as a
  scipy CSR of X's container class in scipy's raw storage order (``dense_output=True``: the dense
  array of it), computed by librp with R resident on the GPU (uploaded once per fitted matrix).
* CSC and dense X are converted to CSR first; sklearn would evaluate those with scipy's CSC or
  dense kernels, whose summation order differs, so those two input kinds match sklearn within
  floating-point reassociation (rtol 1e-5 float32 / 1e-12 float64), not bitwise.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from sklearn.random_projection import SparseRandomProjection as _SkSparseRandomProjection
from sklearn.utils import check_random_state
from sklearn.utils.validation import check_is_fitted, validate_data

from .projector import Projector
from .srp_matrix import check_density, johnson_lindenstrauss_min_dim, sparse_random_matrix

__all__ = ["SparseRandomProjection", "johnson_lindenstrauss_min_dim"]


def _fingerprint(comp, n_sample: int = 4096):
    arrs = [comp.data, comp.indices, comp.indptr] if sp.issparse(comp) else [np.asarray(comp).ravel()]
    fp = [comp.shape, str(comp.dtype)]
    for a in arrs:
        a = np.asarray(a)
        step = max(1, a.size // n_sample)
        fp.append((a.__array_interface__["data"][0], a.size, a[::step].tobytes()))
    return tuple(fp)


class SparseRandomProjection(_SkSparseRandomProjection):
    """``sklearn.random_projection.SparseRandomProjection`` with a GPU ``transform``.

    Extra parameter ``device``: the GPU ordinal R is kept resident on."""

    def __init__(self, n_components="auto", *, density="auto", eps=0.1, dense_output=False,
                 compute_inverse_components=False, random_state=None, device=0):
        super().__init__(n_components=n_components, density=density, eps=eps,
                         dense_output=dense_output,
                         compute_inverse_components=compute_inverse_components,
                         random_state=random_state)
        self.device = device

    def _make_random_matrix(self, n_components, n_features):
        random_state = check_random_state(self.random_state)
        self.density_ = check_density(self.density, n_features)
        return sparse_random_matrix(n_components, n_features, density=self.density_,
                                    random_state=random_state)

    def fit(self, X, y=None):
        self.__dict__.pop("_rp_cache", None)  # a refit always re-uploads R
        return super().fit(X, y)

    def _projector(self) -> Projector:
        """The resident R for the current ``components_``. The cache holds the matrix object itself
        (compared by identity, so a freed-and-reused ``id`` can never alias an older matrix) and a
        fingerprint of its buffers: data pointers, sizes and a strided sample of the values and
        indices, which catches in-place edits of the fitted matrix in the common cases."""
        comp = self.components_
        fp = _fingerprint(comp)
        cached = getattr(self, "_rp_cache", None)
        if cached is None or cached[0] is not comp or cached[1] != fp:
            R = comp.T if sp.issparse(comp) else sp.csr_matrix(np.asarray(comp).T)
            cached = (comp, fp, Projector(R, device=self.device))
            self._rp_cache = cached
        return cached[2]

    def transform(self, X):
        check_is_fitted(self)
        X = validate_data(self, X, accept_sparse=["csr", "csc"], reset=False,
                          dtype=[np.float64, np.float32])
        proj = self._projector()
        if sp.issparse(X):
            Xc = X if X.format == "csr" else X.tocsr()
            out = proj.matmul(Xc)
            if X.format == "csc":
                out = out.tocsc()
        else:
            out = proj.matmul(sp.csr_matrix(X))
            return out.toarray()
        if self.dense_output:
            return out.toarray()
        return out

    def __getstate__(self):
        state = self.__dict__.copy()
        state.pop("_rp_cache", None)
        return state
