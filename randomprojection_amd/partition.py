"""Drop-ins for the reference's partition and row functions, computed on the MI355X.

* ``random_project_mappartitions_function(rdd_row_iterator, local_csr_matrix)`` —
  code/clustermode/randomProjection.py:15-54 (identical copy at code/localmode/randomProjection.py:39-78).
* ``random_project_map_function(feature_vector, local_csr_matrix)`` —
  code/localmode/randomProjection.py:15-36.

Same names, arguments and outputs: rows are duck-typed (``"label" in row``, ``row["id"]``,
``row["label"]``, ``row["features"].{size, indices, values}``), ``local_csr_matrix`` is the m x p
projection operand (any scipy sparse matrix — CSC ``components_.T`` in the recipe — or an already
resident ``Projector``), and the result is a lazy ``zip`` of ``(id, label, SparseVector(p, sorted
int32 indices, float64 values))``. Values are the float32 sums of scipy's csr_matmat upcast to
float64, bit for bit.

What changes (the point of the drop-in): the per-row ``coo_matrix(...).tocsr()`` + ``vstack``
(clustermode:28-43) becomes one vectorised concatenation, R is uploaded once per R object instead
of re-transposed on every call (scipy/_compressed.py:564), and the product and the per-row sort
run on the GPU.

Deliberate differences, documented:
* rows without a ``label`` field: the reference appends a bare id (clustermode:33) and then fails
  with ``TypeError`` in ``i[0]`` (clustermode:53-54); here they yield ``(id, vector)``.
* an empty partition raises ``ValueError("blocks must be 2-D")`` like the reference's ``vstack([])``.
"""
from __future__ import annotations

import numpy as np

from .linalg import SparseVector, Vectors, make_vector
from .linalg import HAVE_PYSPARK as _HAVE_PYSPARK
from .projector import get_projector

__all__ = ["random_project_mappartitions_function", "random_project_map_function", "assemble_rows"]


def assemble_rows(rows):
    """Partition rows -> (ids, labels|None, indptr int64, indices int32, values float32, m).

    Replaces the per-row COO->CSR + vstack of clustermode/randomProjection.py:28-43; values are
    cast with ``astype(np.float32)`` as at :38. Rows are canonicalised (sorted, duplicates summed
    in float32) only if a row is not strictly increasing, which SparseVector rows never are."""
    ids, labels = [], []
    idx_list, val_list, lens = [], [], []
    # bound methods: this loop runs once per row of the partition
    ids_add, labels_add, idx_add, val_add, len_add = (ids.append, labels.append, idx_list.append,
                                                      val_list.append, lens.append)
    asarray, ndarray = np.asarray, np.ndarray
    has_label = False
    m = None
    for row in rows:
        has_label = "label" in row
        ids_add(row["id"])
        labels_add(row["label"] if has_label else None)
        f = row["features"]
        size = f.size
        if size != m:
            if m is None:
                m = int(size)
            elif int(size) != m:
                raise ValueError(f"blocks[{len(ids) - 1},:] has incompatible column dimensions. Got blocks[{len(ids) - 1},:].shape[1] == {size}, expected {m}.")
        ii = f.indices
        if type(ii) is not ndarray:
            ii = asarray(ii)
        vv = f.values
        idx_add(ii)
        val_add(vv if type(vv) is ndarray else asarray(vv))
        len_add(ii.size)
    if not ids:
        raise ValueError("blocks must be 2-D")
    indptr = np.zeros(len(ids) + 1, dtype=np.int64)
    np.cumsum(lens, out=indptr[1:])
    indices = np.concatenate(idx_list).astype(np.int32, copy=False) if indptr[-1] else np.zeros(0, np.int32)
    values = np.concatenate(val_list).astype(np.float32) if indptr[-1] else np.zeros(0, np.float32)
    if indices.size > 1:
        d = np.diff(indices.astype(np.int64))
        starts = indptr[1:-1]
        bad = d <= 0
        bad[starts[(starts >= 1) & (starts - 1 < bad.size)] - 1] = False  # row boundaries
        if bad.any():
            import scipy.sparse as sp

            A = sp.csr_matrix((values, indices, indptr), shape=(len(ids), m))
            A.sum_duplicates()  # what coo_matrix(...).tocsr() does per row
            indptr, indices, values = A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data
    return ids, labels, has_label, indptr, indices, values, m


def random_project_mappartitions_function(rdd_row_iterator, local_csr_matrix):
    """Project one partition of rows (clustermode/randomProjection.py:15-54) on the GPU."""
    ids, labels, has_label, indptr, indices, values, m = assemble_rows(rdd_row_iterator)
    proj = get_projector(local_csr_matrix)
    if m != proj.m:
        raise ValueError(f"matmul: dimension mismatch with signature (n,k={m}),(k={proj.m},m)->(n,m)")
    Cp, Cj, Cx = proj.project_arrays(indptr, indices, values, order="sorted",
                                     out_index_dtype=np.int64)
    p = proj.p
    cj = Cj.astype(np.int32)
    cx = Cx.astype(np.float64)

    def vectors():
        # one vector per row, built lazily as the caller iterates (the reference's zip is lazy too);
        # the constructor is inlined: this loop is most of the partition's host time
        # (boundary 0)
        bounds = Cp.tolist()  # Python ints: cheap per-row slicing
        s = bounds[0]
        if _HAVE_PYSPARK:  # pragma: no cover
            for e in bounds[1:]:
                yield make_vector(p, cj[s:e], cx[s:e])
                s = e
            return
        new, SV = object.__new__, SparseVector
        for e in bounds[1:]:
            v = new(SV)
            v.size = p
            v.indices = cj[s:e]
            v.values = cx[s:e]
            yield v
            s = e

    if has_label:
        return zip(ids, labels, vectors())
    return zip(ids, vectors())


def random_project_map_function(feature_vector, local_csr_matrix):
    """Project one SparseVector (localmode/randomProjection.py:15-36): returns
    ``Vectors.sparse(p, {index: float32 value})`` — sorted indices, float64 storage."""
    proj = get_projector(local_csr_matrix)
    size = int(feature_vector.size)
    if size != proj.m:
        raise ValueError(f"matmul: dimension mismatch with signature (n,k={size}),(k={proj.m},m)->(n,m)")
    idx = np.asarray(feature_vector.indices)
    val = np.asarray(feature_vector.values).astype(np.float32)
    ids, labels, _, indptr, indices, values, _ = assemble_rows(
        [{"id": 0, "features": _Row(size, idx, val)}])
    Cp, Cj, Cx = proj.project_arrays(indptr, indices, values, order="sorted", out_index_dtype=np.int64)
    # the reference casts the row's values to float32 (localmode:34) before SparseVector stores f64
    return Vectors.sparse(proj.p, Cj.astype(np.int32), Cx.astype(np.float32).astype(np.float64))


class _Row:
    __slots__ = ("size", "indices", "values")

    def __init__(self, size, indices, values):
        self.size, self.indices, self.values = size, indices, values
