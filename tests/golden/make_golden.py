"""Generate the committed golden vectors under tests/golden/ (run HERE, never on the GPU box).

Sources of truth, all executed in this container:
* scipy 1.15.3 ``A @ R`` (``_matmul_sparse`` -> ``csr_matmat``): the arithmetic under
  ``code/clustermode/randomProjection.py:46``;
* sklearn 1.7.2 ``SparseRandomProjection(random_state=123).fit`` (``clustermode/randomProjection.py:93-96``);
* the reference module itself, ``code/clustermode/randomProjection.py`` and
  ``code/localmode/randomProjection.py``, imported with ``sys.modules`` stubs for pyspark and
  ``sklearn.externals.joblib`` (importable that way; ``__main__`` not executed).
  Its ``random_project_mappartitions_function`` / ``random_project_map_function`` outputs are stored
  as data (ids, labels, per-row indices and values), never its source.

Usage: python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types
import warnings

import numpy as np
import scipy.sparse as sp

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/code"


# ----------------------------------------------------------------------------- pyspark stubs
class _SparseVector:
    """Mimics pyspark.ml.linalg.SparseVector: pairs are sorted, indices int32, values float64."""

    def __init__(self, size, *args):
        self.size = int(size)
        if len(args) == 1:
            pairs = args[0]
            if isinstance(pairs, dict):
                pairs = pairs.items()
            pairs = sorted(pairs)
            self.indices = np.array([q[0] for q in pairs], dtype=np.int32)
            self.values = np.array([q[1] for q in pairs], dtype=np.float64)
        else:
            self.indices = np.asarray(args[0], dtype=np.int32)
            self.values = np.asarray(args[1], dtype=np.float64)


class _Vectors:
    @staticmethod
    def sparse(size, *args):
        return _SparseVector(size, *args)


def _install_stubs():
    import joblib
    import sklearn.externals as skext

    ps = types.ModuleType("pyspark")
    sql = types.ModuleType("pyspark.sql")
    fn = types.ModuleType("pyspark.sql.functions")
    ty = types.ModuleType("pyspark.sql.types")
    ml = types.ModuleType("pyspark.ml")
    la = types.ModuleType("pyspark.ml.linalg")
    sql.SparkSession = object
    sql.functions = fn
    for n in ["StructType", "StructField", "LongType", "FloatType"]:
        setattr(ty, n, object)
    ty.__all__ = ["StructType", "StructField", "LongType", "FloatType"]
    la.Vectors = _Vectors
    la.VectorUDT = object
    la.SparseVector = _SparseVector
    ps.sql, ps.ml, ml.linalg = sql, ml, la
    sys.modules.update({"pyspark": ps, "pyspark.sql": sql, "pyspark.sql.functions": fn,
                        "pyspark.sql.types": ty, "pyspark.ml": ml, "pyspark.ml.linalg": la,
                        "sklearn.externals.joblib": joblib})
    skext.joblib = joblib


def _load_ref(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# ----------------------------------------------------------------------------- inputs
def kdd_rows(rng, n, m, mean=10.0, values="ones", dtype=np.float32):
    """KDD-shaped CSR: per-row nnz = 1 + Poisson(mean), distinct sorted uniform columns."""
    k = 1 + rng.poisson(mean, size=n)
    k = np.minimum(k, m)
    indptr = np.zeros(n + 1, dtype=np.int64)
    indptr[1:] = np.cumsum(k)
    cols = [np.sort(rng.choice(m, size=int(ki), replace=False)) for ki in k]
    idx = np.concatenate(cols).astype(np.int32) if n else np.zeros(0, np.int32)
    if values == "ones":
        val = np.ones(idx.size, dtype=dtype)
    else:
        val = rng.standard_normal(idx.size).astype(dtype)
    return sp.csr_matrix((val, idx, indptr.astype(np.int32)), shape=(n, m))


def adversarial(R_csr: sp.csr_matrix, rng, dtype=np.float32):
    """Rows that stress scipy's exact semantics: cancellation to an exact 0 (dropped), rounding
    residue of v,v,v,-v,-v,-v (kept), empty rows, duplicate and unsorted input columns, explicit
    zeros, -0.0, NaN/Inf, denormals, and one long row (forces the kernel's heavy-tile path)."""
    m, p = R_csr.shape
    Rc = R_csr.tocsc()
    rows_idx, rows_val = [], []
    # columns k of R touched by >= 6 R rows with one sign
    cand = []
    for k in range(p):
        js = Rc.indices[Rc.indptr[k]:Rc.indptr[k + 1]]
        xs = Rc.data[Rc.indptr[k]:Rc.indptr[k + 1]]
        pos = js[xs > 0]
        if pos.size >= 6:
            cand.append(np.sort(pos[:6]))
        if len(cand) >= 8:
            break
    for c in cand[:4]:
        rows_idx.append(c[:2]); rows_val.append(np.array([0.3, -0.3], dtype))                 # exact 0
        rows_idx.append(c); rows_val.append(np.array([0.1, 0.1, 0.1, -0.1, -0.1, -0.1], dtype))  # residue
        rows_idx.append(c); rows_val.append(np.array([1e-3, 7.0, -7.0, 1e-3, 3.3, -3.3], dtype))
    rows_idx.append(np.zeros(0, np.int64)); rows_val.append(np.zeros(0, dtype))                # empty
    for _ in range(20):
        k = rng.integers(1, 30)
        c = rng.choice(m, size=k, replace=True)        # duplicates + unsorted
        rows_idx.append(c); rows_val.append(rng.standard_normal(k).astype(dtype))
    special = np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1e-40, -1e-42, 3.0e38], dtype)
    for s in special:
        c = np.sort(rng.choice(m, size=12, replace=False))
        v = rng.standard_normal(12).astype(dtype)
        v[rng.integers(0, 12)] = s
        rows_idx.append(c); rows_val.append(v)
    rows_idx.append(np.zeros(0, np.int64)); rows_val.append(np.zeros(0, dtype))
    c = np.sort(rng.choice(m, size=min(m, 6000), replace=False))                               # long row
    rows_idx.append(c); rows_val.append(rng.standard_normal(c.size).astype(dtype))
    indptr = np.zeros(len(rows_idx) + 1, dtype=np.int64)
    indptr[1:] = np.cumsum([len(r) for r in rows_idx])
    A = sp.csr_matrix((np.concatenate(rows_val), np.concatenate(rows_idx).astype(np.int32),
                       indptr.astype(np.int32)), shape=(len(rows_idx), m))
    assert not A.has_canonical_format
    return A


def save_csr(d, prefix, M):
    d[prefix + "_indptr"] = M.indptr
    d[prefix + "_indices"] = M.indices
    d[prefix + "_data"] = M.data
    d[prefix + "_shape"] = np.array(M.shape, dtype=np.int64)


def product(A, R):
    C = A @ R        # scipy raw order
    assert sp.isspmatrix_csr(C)
    return C


def main():
    from sklearn.random_projection import SparseRandomProjection

    rng = np.random.default_rng(2012)
    out = {}

    # R1: KDD recipe shape scaled down (tracking-selection branch), f32 fit as in the recipe
    m1, p1 = 100_000, 256
    srp1 = SparseRandomProjection(n_components=p1, random_state=123).fit(
        sp.csr_matrix((10, m1), dtype=np.float32))
    C1 = srp1.components_.copy()
    save_csr(out, "comp1", C1)                  # raw sklearn storage (unsorted rows), f32
    R1 = srp1.components_.T.astype(np.float32)  # clustermode/randomProjection.py:101 (CSC)
    # R2: permutation branch (m < 1e4), f64 fit
    m2, p2 = 5000, 64
    srp2 = SparseRandomProjection(n_components=p2, random_state=123).fit(
        sp.csr_matrix((10, m2), dtype=np.float64))
    save_csr(out, "comp2", srp2.components_)
    R2 = srp2.components_.T                     # CSC f64

    cases = {
        "kdd_ones": (kdd_rows(rng, 2000, m1), R1),
        "kdd_vals": (kdd_rows(rng, 2000, m1, values="normal"), R1),
        "adv_f32": (adversarial(sp.csr_matrix(R1), rng), R1),
        "vals_f64": (kdd_rows(rng, 1500, m2, mean=30, values="normal", dtype=np.float64), R2),
        "mixed_f32xf64": (kdd_rows(rng, 1500, m2, mean=30, values="normal"), R2),
        "adv_f64": (adversarial(sp.csr_matrix(R2), rng, dtype=np.float64), R2),
    }
    names = []
    for name, (A, R) in cases.items():
        C = product(A, R)
        save_csr(out, "A_" + name, A)
        save_csr(out, "C_" + name, C)
        Cs = C.copy()
        Cs.sort_indices()
        out["Csorted_" + name + "_indices"] = Cs.indices
        out["Csorted_" + name + "_data"] = Cs.data
        out["R_" + name] = np.array([1 if R is R1 else 2])
        names.append(name)
        print(f"{name}: A {A.shape} nnz={A.nnz} C nnz={C.nnz} dtype={C.dtype} idx={C.indices.dtype}")
    out["cases"] = np.array(names)

    # the reference's own functions, stub-imported, on rows of kdd_vals
    _install_stubs()
    cm = _load_ref(os.path.join(REF, "clustermode", "randomProjection.py"), "ref_clustermode")
    lm = _load_ref(os.path.join(REF, "localmode", "randomProjection.py"), "ref_localmode")
    A = cases["kdd_vals"][0][:300]
    rows = []
    for i in range(A.shape[0]):
        s, e = A.indptr[i], A.indptr[i + 1]
        rows.append({"id": 1000 + 7 * i, "label": float(i % 2),
                     "features": _SparseVector(m1, A.indices[s:e], A.data[s:e].astype(np.float64))})
    res = list(cm.random_project_mappartitions_function(iter(rows), R1))
    lres = list(lm.random_project_mappartitions_function(iter(rows), R1))
    assert len(res) == len(rows)
    ptr = [0]
    for (a, b, v), (a2, b2, v2) in zip(res, lres):
        assert a == a2 and b == b2 and np.array_equal(v.indices, v2.indices) and np.array_equal(v.values, v2.values)
        ptr.append(ptr[-1] + len(v.indices))
    out["ref_part_ids"] = np.array([r[0] for r in res], dtype=np.int64)
    out["ref_part_labels"] = np.array([r[1] for r in res], dtype=np.float64)
    out["ref_part_indptr"] = np.array(ptr, dtype=np.int64)
    out["ref_part_indices"] = np.concatenate([r[2].indices for r in res]).astype(np.int32)
    out["ref_part_values"] = np.concatenate([r[2].values for r in res]).astype(np.float64)
    out["ref_part_size"] = np.array([res[0][2].size])
    # single-row map variant (localmode/randomProjection.py:15-36) on 40 rows
    mptr, midx, mval = [0], [], []
    for r in rows[:40]:
        v = lm.random_project_map_function(r["features"], R1)
        midx.append(v.indices)
        mval.append(v.values)
        mptr.append(mptr[-1] + len(v.indices))
    out["ref_map_indptr"] = np.array(mptr, dtype=np.int64)
    out["ref_map_indices"] = np.concatenate(midx).astype(np.int32)
    out["ref_map_values"] = np.concatenate(mval).astype(np.float64)
    # the reference's no-label branch (clustermode/randomProjection.py:33,53-54) raises
    try:
        list(cm.random_project_mappartitions_function(iter([{"id": 1, "features": rows[0]["features"]}]), R1))
        out["ref_nolabel_raises"] = np.array([0])
    except TypeError:
        out["ref_nolabel_raises"] = np.array([1])
    try:
        cm.random_project_mappartitions_function(iter([]), R1)
        out["ref_empty_raises"] = np.array([0])
    except ValueError:
        out["ref_empty_raises"] = np.array([1])

    path = os.path.join(HERE, "golden_v1.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
