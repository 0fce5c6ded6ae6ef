"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/smmp.c header).

Python face of the CPU restatement of scipy's ``csr_matmat_maxnnz`` + ``csr_matmat`` — the
arithmetic under ``features_matrix.dot(local_csr_matrix)`` at
``code/clustermode/randomProjection.py:46`` (scipy/sparse/_compressed.py:546-604).

* ``matmat(A, B)``        — C restatement (oracle/smmp.c) through ctypes; returns the raw
                             (indptr, indices, data) in scipy's storage order.
* ``matmat_py(A, B)``     — the same algorithm as pure-Python loops, for small cases only; used to
                             cross-check the C build.
* ``project_mt(...)``      — multi-threaded C driver, the bench's CPU baseline (kind "port").
* ``partition_function_py`` — restatement of the reference partition function
  (``clustermode/randomProjection.py:15-54``) on top of ``matmat`` (per-row sorted output, f64
  values), used as the checker for the drop-in.

Parity: pinned against scipy 1.15.3 golden vectors (tests/golden/, tests/test_oracle.py).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_SMMP_LIB: another build of the same source (tests/sanitize: the ASan/UBSan one)
_LIB_PATH = os.environ.get("ORACLE_SMMP_LIB") or os.path.join(_HERE, "build", "liboracle_smmp.so")
_lib = None


def build() -> str:
    """Compile oracle/smmp.c with the committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        for sfx in ("i32_f32", "i32_f64", "i64_f32", "i64_f64"):
            f = getattr(lib, "oracle_maxnnz_" + sfx)
            f.restype = i64
            f.argtypes = [i64, i64, vp, vp, vp, vp]
            g = getattr(lib, "oracle_matmat_" + sfx)
            g.restype = i64
            g.argtypes = [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        lib.oracle_project_mt_i32_f32.restype = i64
        lib.oracle_project_mt_i32_f32.argtypes = [i64, i64, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        _lib = lib
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _operands(A, B):
    """scipy's operand preparation in ``_matmul_sparse``: B converted to CSR (``self.__class__``),
    index dtype = int64 if any index array is int64 (``get_index_dtype``, check_contents=False),
    value dtype = ``upcast(A.dtype, B.dtype)``."""
    import scipy.sparse as sp

    A = sp.csr_matrix(A)
    B = sp.csr_matrix(B)
    if A.shape[1] != B.shape[0]:
        raise ValueError("matmul: dimension mismatch")
    idx = np.int64 if any(a.dtype == np.int64 for a in (A.indptr, A.indices, B.indptr, B.indices)) else np.int32
    T = np.result_type(A.dtype, B.dtype)
    if T not in (np.float32, np.float64):
        T = np.dtype(np.float64)
    return A, B, np.dtype(idx), np.dtype(T)


def matmat(A, B, index_dtype=None):
    """C @ in scipy's raw order: returns (indptr, indices, data, shape)."""
    lib = _load()
    A, B, idx, T = _operands(A, B)
    if index_dtype is not None:
        idx = np.dtype(index_dtype)
    sfx = ("i64" if idx == np.int64 else "i32") + "_" + ("f64" if T == np.float64 else "f32")
    M, N = A.shape[0], B.shape[1]
    Ap = np.ascontiguousarray(A.indptr, dtype=idx)
    Aj = np.ascontiguousarray(A.indices, dtype=idx)
    Bp = np.ascontiguousarray(B.indptr, dtype=idx)
    Bj = np.ascontiguousarray(B.indices, dtype=idx)
    Ax = np.ascontiguousarray(A.data, dtype=T)
    Bx = np.ascontiguousarray(B.data, dtype=T)
    cap = getattr(lib, "oracle_maxnnz_" + sfx)(M, N, _ptr(Ap), _ptr(Aj), _ptr(Bp), _ptr(Bj))
    if cap < 0:
        raise MemoryError("oracle maxnnz allocation failed")
    out_idx = np.int64 if cap > np.iinfo(np.int32).max else idx
    if out_idx != idx:  # recompute with 64-bit indices, as scipy re-derives idx_dtype with maxval=nnz
        return matmat(A, B, index_dtype=np.int64)
    Cp = np.empty(M + 1, dtype=idx)
    Cj = np.empty(max(cap, 1), dtype=idx)
    Cx = np.empty(max(cap, 1), dtype=T)
    nnz = getattr(lib, "oracle_matmat_" + sfx)(M, N, _ptr(Ap), _ptr(Aj), _ptr(Ax), _ptr(Bp), _ptr(Bj),
                                                _ptr(Bx), _ptr(Cp), _ptr(Cj), _ptr(Cx))
    if nnz < 0:
        raise MemoryError("oracle matmat allocation failed")
    return Cp, Cj[:nnz].copy(), Cx[:nnz].copy(), (M, N), cap


def matmat_py(A, B):
    """Pure-Python loop restatement of csr_matmat (small inputs only)."""
    A, B, idx, T = _operands(A, B)
    T = T.type
    M, N = A.shape[0], B.shape[1]
    nxt = [-1] * N
    sums = [T(0)] * N
    Cp, Cj, Cx = [0], [], []
    Ap, Aj, Ax = A.indptr, A.indices, A.data.astype(T)
    Bp, Bj, Bx = B.indptr, B.indices, B.data.astype(T)
    with np.errstate(all="ignore"):
        for i in range(M):
            head, length = -2, 0
            for jj in range(Ap[i], Ap[i + 1]):
                j, v = Aj[jj], Ax[jj]
                for kk in range(Bp[j], Bp[j + 1]):
                    k = int(Bj[kk])
                    sums[k] = T(sums[k] + T(v * Bx[kk]))
                    if nxt[k] == -1:
                        nxt[k] = head
                        head = k
                        length += 1
            for _ in range(length):
                if sums[head] != 0:
                    Cj.append(head)
                    Cx.append(sums[head])
                t = head
                head = nxt[head]
                nxt[t] = -1
                sums[t] = T(0)
            Cp.append(len(Cj))
    return (np.asarray(Cp, dtype=idx), np.asarray(Cj, dtype=idx), np.asarray(Cx, dtype=T), (M, N))


def project_mt(Ap, Aj, Ax, Bp, Bj, Bx, n_col, n_threads):
    """Threaded C driver over int32/f32 CSR operands (bench cpu_baseline). Returns total nnz."""
    lib = _load()
    Ap = np.ascontiguousarray(Ap, dtype=np.int32)
    Aj = np.ascontiguousarray(Aj, dtype=np.int32)
    Ax = np.ascontiguousarray(Ax, dtype=np.float32)
    Bp = np.ascontiguousarray(Bp, dtype=np.int32)
    Bj = np.ascontiguousarray(Bj, dtype=np.int32)
    Bx = np.ascontiguousarray(Bx, dtype=np.float32)
    n = lib.oracle_project_mt_i32_f32(len(Ap) - 1, n_col, _ptr(Ap), _ptr(Aj), _ptr(Ax), _ptr(Bp), _ptr(Bj),
                                      _ptr(Bx), int(n_threads))
    if n < 0:
        raise MemoryError("oracle_project_mt failed")
    return n


def sorted_rows(indptr, indices, data):
    """Per-row ascending-index form (what pyspark's SparseVector makes of each row, a6)."""
    indptr = np.asarray(indptr, dtype=np.int64)
    n = len(indptr) - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    order = np.lexsort((np.asarray(indices), rows))
    return np.asarray(indices)[order], np.asarray(data)[order]


def partition_function_py(rows, R):
    """Restatement of ``random_project_mappartitions_function`` (clustermode/randomProjection.py:15-54)
    as a checker: per-row features -> CSR (f32 values), ``@ R`` through ``matmat``, per-row output
    sorted by index with values upcast to f64. Returns a list of ``(id, label, idx, vals)`` or
    ``(id, idx, vals)`` tuples (the no-label branch as the drop-in defines it)."""
    import scipy.sparse as sp

    rows = list(rows)
    if not rows:
        raise ValueError("blocks must be 2-D")
    m = rows[0]["features"].size
    indptr = [0]
    idx, val = [], []
    for r in rows:
        f = r["features"]
        idx.append(np.asarray(f.indices, dtype=np.int32))
        val.append(np.asarray(f.values).astype(np.float32))
        indptr.append(indptr[-1] + len(f.indices))
    A = sp.csr_matrix((np.concatenate(val), np.concatenate(idx), np.asarray(indptr)), shape=(len(rows), m))
    A.sum_duplicates()
    Cp, Cj, Cx, _, _ = matmat(A, R)
    out = []
    for i, r in enumerate(rows):
        j = Cj[Cp[i]:Cp[i + 1]]
        x = Cx[Cp[i]:Cp[i + 1]]
        o = np.argsort(j, kind="stable")
        jj = j[o].astype(np.int32)
        xx = x[o].astype(np.float64)
        if "label" in rows[-1]:
            out.append((r["id"], r["label"], jj, xx))
        else:
            out.append((r["id"], jj, xx))
    return out
