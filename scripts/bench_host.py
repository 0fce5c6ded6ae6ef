"""Host-boundary benchmarks (SURVEY.md §8(d) boundaries 2 and the drop-in):
  * host CSR in -> GPU -> host CSR out (PCIe-inclusive), Projector.matmul on KDD-shaped rows;
  * the drop-in random_project_mappartitions_function on Row-like dicts (Python objects in and
    out, as Spark hands them over), next to the oracle's restatement of the reference recipe
    (per-row rows -> CSR, scipy-kernel restatement, SparseVector-like output) on one core.
Prints one JSON line. Not the headline metric (bench.py is).

    python scripts/bench_host.py [--rows 1000000] [--part-rows 100000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def kdd_csr(rng, n, m):
    k = 1 + rng.poisson(10, n)
    cols = rng.integers(0, m, size=int(k.sum()), dtype=np.int64)
    indptr = np.concatenate([[0], np.cumsum(k)])
    # sort + dedupe within rows (vectorised): sort by (row, col), drop repeats
    rows = np.repeat(np.arange(n), k)
    order = np.lexsort((cols, rows))
    rows, cols = rows[order], cols[order]
    keep = np.ones(cols.size, bool)
    keep[1:] = (rows[1:] != rows[:-1]) | (cols[1:] != cols[:-1])
    rows, cols = rows[keep], cols[keep]
    indptr = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.int32)
    return sp.csr_matrix((np.ones(cols.size, np.float32), cols.astype(np.int32), indptr), shape=(n, m))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--part-rows", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import torch  # noqa: F401  (one HIP runtime; see _native.load)

    from oracle import smmp
    from randomprojection_amd import Projector, random_project_mappartitions_function, srp_matrix as sm
    from randomprojection_amd.linalg import SparseVector

    R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
    P = Projector(R)
    rng = np.random.default_rng(2012)
    A = kdd_csr(rng, args.rows, sm.KDD_M)
    P.matmul(A[:1000])
    t = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        C = P.matmul(A)
        t.append(time.perf_counter() - t0)
    host_rows_s = args.rows / min(t)

    B = A[: args.part_rows]
    rows = [{"id": i, "label": float(i & 1),
             "features": SparseVector(sm.KDD_M, B.indices[B.indptr[i]:B.indptr[i + 1]],
                                      B.data[B.indptr[i]:B.indptr[i + 1]].astype(np.float64))}
            for i in range(B.shape[0])]
    t0 = time.perf_counter()
    out = list(random_project_mappartitions_function(iter(rows), R))
    dropin_s = time.perf_counter() - t0
    assert len(out) == len(rows)
    n_ref = min(args.part_rows, 20_000)
    t0 = time.perf_counter()
    smmp.partition_function_py(rows[:n_ref], R)
    ref_s = (time.perf_counter() - t0) * args.part_rows / n_ref
    print(json.dumps({
        "boundary": "host CSR in -> host CSR out (PCIe-inclusive)",
        "rows": args.rows, "host_rows_per_s": host_rows_s, "nnz_out": int(C.nnz),
        "dropin_partition": {"rows": args.part_rows, "rows_per_s": args.part_rows / dropin_s,
                             "us_per_row": dropin_s / args.part_rows * 1e6},
        "recipe_restatement_1core": {"rows_per_s": args.part_rows / ref_s, "us_per_row": ref_s / args.part_rows * 1e6,
                                     "note": "oracle.smmp.partition_function_py: row dicts -> CSR -> C scipy-kernel restatement -> sorted f64 rows, 1 core"},
    }))


if __name__ == "__main__":
    main()
