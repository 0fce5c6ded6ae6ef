"""Recipe-faithful CPU restatement of the reference's partition function — TEST/BENCH
INFRASTRUCTURE ONLY (the CPU baseline of SURVEY.md §8(d)(i)); never imported by the product.

Restates ``random_project_mappartitions_function`` of code/clustermode/randomProjection.py:15-54
step for step with the same scipy operations, so that its cost is the reference's cost:
  * per row (:28-40): ``"label" in row`` key capture, ``values.astype(np.float32)``, a 1 x m
    ``coo_matrix((data, (row_indices, col_indices))).tocsr()``;
  * ``vstack`` of the single-row matrices (:42);
  * ``features_matrix.dot(local_csr_matrix)`` (:45) — scipy converts the CSC operand to CSR on
    every call (scipy/sparse/_compressed.py:564) and runs csr_matmat;
  * per output row ``Vectors.sparse(PROJECT_DIM_SIZE, zip(i.indices, i.data))`` (:49-50), iterating
    the CSR result row by row; pyspark's Vectors.sparse is stood in by the package's pyspark-shaped
    SparseVector (sorts the pairs, int32 indices, float64 values).
Returns a list (the reference returns a lazy zip; materialising it is what Spark does with it).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as ssp


def recipe_partition(rows, local_csr_matrix, vectors_sparse=None):
    if vectors_sparse is None:
        from randomprojection_amd.linalg import Vectors

        vectors_sparse = Vectors.sparse
    keys = []
    singles = []
    p = local_csr_matrix.shape[1]
    row = None
    for row in rows:
        keys.append((row["id"], row["label"]) if "label" in row else (row["id"]))
        f = row["features"]
        col_indices = f.indices
        data = f.values.astype(np.float32)
        singles.append(ssp.coo_matrix((data, ([0] * len(col_indices), col_indices)), shape=(1, f.size)).tocsr())
    features = ssp.vstack(singles)
    del singles
    projected = features.dot(local_csr_matrix)
    vecs = [vectors_sparse(p, zip(i.indices, i.data)) for i in projected]
    if row is not None and "label" in row:
        return list(zip((k[0] for k in keys), (k[1] for k in keys), vecs))
    return list(zip(keys, vecs))
