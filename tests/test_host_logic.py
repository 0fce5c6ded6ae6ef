"""Host-side logic of the drop-ins that needs no GPU."""
import numpy as np
import pytest

from randomprojection_amd.linalg import SparseVector, Vectors
from randomprojection_amd.partition import assemble_rows, random_project_mappartitions_function
from randomprojection_amd.projector import scipy_result_index_dtype


def _rows(n, m=1000, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = rng.integers(0, 12)
        idx = np.sort(rng.choice(m, size=k, replace=False))
        out.append({"id": i, "label": float(i % 2), "features": SparseVector(m, idx, rng.standard_normal(k))})
    return out


def test_assemble_rows_matches_vstack():
    import scipy.sparse as ssp
    rows = _rows(50)
    ids, labels, has_label, indptr, indices, values, m = assemble_rows(iter(rows))
    ref = ssp.vstack([ssp.coo_matrix((r["features"].values.astype(np.float32),
                                      ([0] * len(r["features"].indices), r["features"].indices)),
                                     shape=(1, m)).tocsr() for r in rows])
    assert has_label and ids == list(range(50)) and m == 1000
    assert np.array_equal(indptr, ref.indptr) and np.array_equal(indices, ref.indices)
    assert np.array_equal(values, ref.data) and values.dtype == np.float32


def test_assemble_rows_canonicalises_unsorted_duplicates():
    class F:
        size = 10
        indices = np.array([5, 2, 5])
        values = np.array([1.0, 2.0, 3.0])
    _, _, _, indptr, indices, values, _ = assemble_rows([{"id": 1, "features": F()}])
    assert list(indices) == [2, 5] and list(values) == [2.0, 4.0]


def test_empty_partition_raises_like_reference():
    with pytest.raises(ValueError, match="blocks must be 2-D"):
        random_project_mappartitions_function(iter([]), None)


def test_mismatched_row_sizes_raise():
    rows = _rows(3)
    rows[1]["features"] = SparseVector(999, [1], [1.0])
    with pytest.raises(ValueError):
        assemble_rows(rows)


def test_sparse_vector_semantics():
    v = Vectors.sparse(8, zip([5, 1, 3], [0.5, 1.5, 2.5]))
    assert list(v.indices) == [1, 3, 5] and v.values.dtype == np.float64
    assert v.toArray()[3] == 2.5 and v.numNonzeros() == 3
    with pytest.raises(TypeError):
        SparseVector(8, [3, 1], [1.0, 2.0])


def test_result_index_dtype_rule():
    i32, i64 = np.zeros(2, np.int32), np.zeros(2, np.int64)
    assert scipy_result_index_dtype((i32, i32), 10) == np.int32
    assert scipy_result_index_dtype((i32, i64), 10) == np.int64
    assert scipy_result_index_dtype((i32, i32), 2**31) == np.int64


def test_hostmem_pool_recycles_only_dead_arrays(monkeypatch):
    """Pooled result arrays (hostmem.empty) are plain numpy arrays; a mapping goes back to the pool
    only after the array and every view of it are gone, and idle memory is bounded."""
    import gc
    from randomprojection_amd import hostmem

    a = hostmem.empty(3_000_000, np.int32)
    assert a.shape == (3_000_000,) and a.dtype == np.int32 and a.flags.writeable and a.flags.c_contiguous
    a[:] = 5
    v = a[100:200]
    addr = a.ctypes.data
    del a
    gc.collect()
    b = hostmem.empty(3_000_000, np.int32)          # the first mapping is still held by v
    assert b.ctypes.data != addr and np.all(v == 5)
    del v
    gc.collect()
    c = hostmem.empty(2_800_000, np.float32)        # best fit: the recycled mapping
    assert c.ctypes.data == addr
    assert hostmem.empty(10, np.int64).shape == (10,)   # small requests: np.empty
    monkeypatch.setenv("RP_HOST_POOL_BYTES", "0")
    del b, c
    gc.collect()
    st = hostmem.pool_stats()
    assert st["idle_bytes"] == 0 and st["unmapped"] >= 2
