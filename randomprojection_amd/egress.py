"""Output egress of projected partitions.

The reference turns each projected partition into ``(id, label, SparseVector(p, ...))`` rows
(code/clustermode/randomProjection.py:49-52), builds a DataFrame with
``train_schema = (id Long not null, label Float not null, features VectorUDT not null)``
(clustermode:75-80, ``.toDF(train_schema)`` at :110) and writes Parquet (:113).

Here the projected CSR goes straight to Parquet with pyarrow, columnar, no per-row objects:
``features`` is stored as Spark's VectorUDT storage struct
``{type: int8 (0 = sparse), size: int32, indices: list<int32>, values: list<float64>}`` and the
Spark schema JSON is put under ``org.apache.spark.sql.parquet.row.metadata`` so Spark reads the
column back as ``VectorUDT``. Parity with Spark's own writer is unpinned (no JVM here); the
layout restates Spark's published ``VectorUDT.sqlType``.
"""
from __future__ import annotations

import json

import numpy as np
import scipy.sparse as sp

from .linalg import make_vector

__all__ = ["rows", "write_parquet", "read_parquet", "SPARK_SCHEMA_JSON"]

_VECTOR_SQLTYPE = {
    "type": "struct",
    "fields": [
        {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
        {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
        {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
         "nullable": True, "metadata": {}},
        {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
         "nullable": True, "metadata": {}},
    ],
}
SPARK_SCHEMA_JSON = json.dumps({
    "type": "struct",
    "fields": [
        {"name": "id", "type": "long", "nullable": False, "metadata": {}},
        {"name": "label", "type": "float", "nullable": False, "metadata": {}},
        {"name": "features", "type": {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT",
                                      "pyClass": "pyspark.ml.linalg.VectorUDT", "sqlType": _VECTOR_SQLTYPE},
         "nullable": False, "metadata": {}},
    ],
})


def _sorted_csr(C) -> sp.csr_matrix:
    C = sp.csr_matrix(C)
    if not C.has_sorted_indices:
        C = C.copy()
        C.sort_indices()
    return C


def rows(ids, labels, C):
    """Lazy ``(id, label, SparseVector)`` tuples (clustermode:49-52), indices ascending, f64 values."""
    C = _sorted_csr(C)
    cj = C.indices.astype(np.int32, copy=False)
    cx = C.data.astype(np.float64)
    for i in range(C.shape[0]):
        s, e = C.indptr[i], C.indptr[i + 1]
        yield ids[i], labels[i], make_vector(C.shape[1], cj[s:e], cx[s:e])


_MAX_LIST_ENTRIES = 2**31 - 1  # Arrow list<...> offsets are int32


def _row_slices(indptr, limit=_MAX_LIST_ENTRIES):
    """[r0, r1) row ranges whose entries each fit one Arrow list array (int32 offsets)."""
    n, out, r0 = len(indptr) - 1, [], 0
    while r0 < n or not out:
        r1 = int(np.searchsorted(indptr, indptr[r0] + limit, side="right")) - 1
        r1 = max(r1, r0 + 1) if n else 0
        if r1 > n:
            r1 = n
        if r1 - r0 == 1 and indptr[r1] - indptr[r0] > limit:
            raise ValueError("one row holds more than 2^31 - 1 entries")
        out.append((r0, r1))
        r0 = r1
        if n == 0:
            break
    return out


def _table(ids, labels, C):
    """The partition as a pyarrow Table; a partition past 2^31 - 1 output entries becomes several
    record batches (each with its own int32 list offsets), never a silently wrapped offset."""
    import pyarrow as pa

    C = _sorted_csr(C)
    if C.nnz <= _MAX_LIST_ENTRIES:
        return _table_part(ids, labels, C)
    parts = [_table_part(ids[a:b], labels[a:b], C[a:b]) for a, b in _row_slices(np.asarray(C.indptr, np.int64))]
    return pa.concat_tables(parts)


def _table_part(ids, labels, C):
    import pyarrow as pa

    n, p = C.shape
    assert C.nnz <= _MAX_LIST_ENTRIES
    offs = pa.array(np.asarray(C.indptr, dtype=np.int64) - int(C.indptr[0])).cast(pa.int32())
    it = pa.list_(pa.field("element", pa.int32(), nullable=False))
    vt = pa.list_(pa.field("element", pa.float64(), nullable=False))
    idx = pa.ListArray.from_arrays(offs, pa.array(C.indices.astype(np.int32, copy=False)), type=it)
    val = pa.ListArray.from_arrays(offs, pa.array(C.data.astype(np.float64)), type=vt)
    feat = pa.StructArray.from_arrays(
        [pa.array(np.zeros(n, np.int8)), pa.array(np.full(n, p, np.int32)), idx, val],
        fields=[pa.field("type", pa.int8(), nullable=False), pa.field("size", pa.int32()),
                pa.field("indices", it), pa.field("values", vt)])
    schema = pa.schema([pa.field("id", pa.int64(), nullable=False),
                        pa.field("label", pa.float32(), nullable=False),
                        pa.field("features", feat.type, nullable=False)],
                       metadata={"org.apache.spark.sql.parquet.row.metadata": SPARK_SCHEMA_JSON})
    return pa.Table.from_arrays([pa.array(np.asarray(ids, dtype=np.int64)),
                                 pa.array(np.asarray(labels, dtype=np.float32)), feat], schema=schema)


def write_parquet(path, ids, labels, C, compression: str = "snappy"):
    """Write one projected partition (``part-*.parquet`` of the reference's output directory)."""
    import pyarrow.parquet as pq

    if C.shape[0] != len(ids) or len(ids) != len(labels):
        raise ValueError("ids, labels and C must have the same number of rows")
    pq.write_table(_table(ids, labels, C), path, compression=compression)


def read_parquet(path):
    """-> (ids int64, labels float32, C csr float64) from a file written by ``write_parquet``."""
    import pyarrow.parquet as pq

    t = pq.read_table(path)
    ids = t.column("id").to_numpy()
    labels = t.column("label").to_numpy()
    f = t.column("features").combine_chunks()
    size = int(f.field("size")[0].as_py()) if len(f) else 0
    idx, val = f.field("indices"), f.field("values")
    indptr = idx.offsets.to_numpy().astype(np.int64)
    C = sp.csr_matrix((val.values.to_numpy(), idx.values.to_numpy(), indptr - indptr[0]), shape=(len(ids), size))
    return ids, labels, C
