"""``Vectors.sparse`` / ``SparseVector`` as the drop-ins emit them.

The reference emits ``pyspark.ml.linalg.Vectors.sparse(p, zip(indices, data))``
(code/clustermode/randomProjection.py:49-50) and ``Vectors.sparse(ndim, dict(...))``
(code/localmode/randomProjection.py:36): pyspark sorts the pairs, stores int32 indices and float64
values. When pyspark is importable the drop-ins build real pyspark vectors; otherwise this
minimal class with the same fields and ordering rules stands in (no JVM needed).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - pyspark is not installed in this image
    from pyspark.ml.linalg import SparseVector as _PySparkVector  # type: ignore
    from pyspark.ml.linalg import Vectors as _PySparkVectors  # type: ignore
except Exception:  # noqa: BLE001
    _PySparkVector = None
    _PySparkVectors = None

__all__ = ["SparseVector", "Vectors", "HAVE_PYSPARK"]
HAVE_PYSPARK = _PySparkVector is not None


class SparseVector:
    """Sparse vector of dimension ``size`` with strictly increasing int32 ``indices`` and
    float64 ``values`` (pyspark.ml.linalg.SparseVector semantics)."""

    __slots__ = ("size", "indices", "values")

    def __init__(self, size, *args):
        self.size = int(size)
        if len(args) == 1:
            pairs = args[0]
            if isinstance(pairs, dict):
                pairs = pairs.items()
            pairs = sorted(pairs)
            self.indices = np.array([q[0] for q in pairs], dtype=np.int32)
            self.values = np.array([q[1] for q in pairs], dtype=np.float64)
        elif len(args) == 2:
            self.indices = np.asarray(args[0], dtype=np.int32)
            self.values = np.asarray(args[1], dtype=np.float64)
            if self.indices.size > 1 and np.any(np.diff(self.indices) <= 0):
                raise TypeError("Indices are not strictly increasing")
        else:
            raise TypeError("SparseVector(size, pairs) or SparseVector(size, indices, values)")
        if self.indices.size != self.values.size:
            raise ValueError("indices and values must have the same length")

    @classmethod
    def _trusted(cls, size, indices, values):
        v = cls.__new__(cls)
        v.size = int(size)
        v.indices = indices
        v.values = values
        return v

    def numNonzeros(self):
        return int(np.count_nonzero(self.values))

    def toArray(self):
        a = np.zeros(self.size, dtype=np.float64)
        a[self.indices] = self.values
        return a

    def __len__(self):
        return self.size

    def __eq__(self, other):
        return (hasattr(other, "indices") and self.size == getattr(other, "size", None)
                and np.array_equal(self.indices, np.asarray(other.indices))
                and np.array_equal(self.values, np.asarray(other.values)))

    def __repr__(self):
        return f"SparseVector({self.size}, {dict(zip(self.indices.tolist(), self.values.tolist()))})"


class Vectors:
    @staticmethod
    def sparse(size, *args):
        if _PySparkVectors is not None:  # pragma: no cover
            return _PySparkVectors.sparse(size, *args)
        return SparseVector(size, *args)


_new_vector = SparseVector.__new__


def make_vector(size, indices_sorted_i32, values_f64):
    """Vector from already sorted, deduplicated arrays (the GPU emits rows in ascending order)."""
    if _PySparkVector is not None:  # pragma: no cover
        return _PySparkVector(size, indices_sorted_i32, values_f64)
    v = _new_vector(SparseVector)
    v.size = size
    v.indices = indices_sorted_i32
    v.values = values_f64
    return v
