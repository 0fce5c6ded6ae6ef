"""CPU reference timed beside the GPU line — TEST/BENCH INFRASTRUCTURE ONLY.

bench.py runs this as a CHILD process (no GPU state in it, so it may fork workers) on a bounded
sample of the same synthetic workload, saved by bench.py as .npy files in a scratch directory:

  (i)  the recipe restated (oracle/recipe.py = code/clustermode/randomProjection.py:15-54 step for
       step: per-row COO -> CSR, vstack, CSR @ CSC R with scipy's per-call conversion, sorted
       per-row SparseVector output), one process per core on its own partition of `part_rows`
       rows (Spark local[N]'s one task per core), plus the same on one core;
  (ii) scipy's kernel pair alone (csr_matmat_maxnnz + csr_matmat, oracle/smmp.c restating it,
       bit-identical by fixture test) on N threads over `kernel_rows` rows, plus one thread.

Cores: the CPUs this process may run on (os.sched_getaffinity), capped by the cgroup CPU quota
(/sys/fs/cgroup/cpu.max) when one is set, since threads beyond the quota only time-slice; both
numbers are reported.

    python -m oracle.cpu_baseline <dir> <m> <part_rows> <kernel_rows>   -> one JSON line
"""
from __future__ import annotations

import json
import math
import multiprocessing as mp
import os
import sys
import time

import numpy as np
import scipy.sparse as ssp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_G = {}  # worker inputs, inherited through fork


def usable_cores():
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(math.floor(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def _rows(ap, aj, ax, m, lo, hi):
    """The partition's rows as the recipe receives them (Row-like dicts with a SparseVector)."""
    from randomprojection_amd.linalg import SparseVector

    return [{"id": i, "label": float(i & 1),
             "features": SparseVector(m, aj[ap[i]:ap[i + 1]], ax[ap[i]:ap[i + 1]].astype(np.float64))}
            for i in range(lo, hi)]


def _recipe_worker(k):
    from oracle.recipe import recipe_partition

    g = _G
    lo = k * g["part"]
    rows = _rows(g["ap"], g["aj"], g["ax"], g["m"], lo, lo + g["part"])
    g["barrier"].wait()
    t0 = time.perf_counter()
    out = recipe_partition(rows, g["Rcsc"])
    dt = time.perf_counter() - t0
    assert len(out) == len(rows)
    return dt


def main():
    d, m, part, krows = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    ap = np.load(os.path.join(d, "ap.npy"))
    aj = np.load(os.path.join(d, "aj.npy"))
    ax = np.load(os.path.join(d, "ax.npy"))
    Rp = np.load(os.path.join(d, "rp.npy"))
    Rj = np.load(os.path.join(d, "rj.npy"))
    Rx = np.load(os.path.join(d, "rx.npy"))
    p = int(np.load(os.path.join(d, "p.npy")))
    n = ap.size - 1
    cores, aff, quota = usable_cores()
    res = {"cores": cores, "affinity_cpus": aff, "cgroup_quota_cpus": quota}

    # (ii) kernel restatement, N threads and 1 thread
    from oracle import smmp

    kr = min(krows, n)
    ap32 = ap[:kr + 1].astype(np.int32)
    smmp.project_mt(ap32[:1001], aj, ax, Rp, Rj, Rx, p, 1)  # warm
    t0 = time.perf_counter()
    smmp.project_mt(ap32, aj, ax, Rp, Rj, Rx, p, cores)
    dt_n = time.perf_counter() - t0
    k1 = max(1000, kr // max(cores, 1))
    t0 = time.perf_counter()
    smmp.project_mt(ap32[:k1 + 1], aj, ax, Rp, Rj, Rx, p, 1)
    dt_1 = time.perf_counter() - t0
    res["kernel_port"] = {"value": kr / dt_n, "rows": kr, "threads": cores, "wall_s": dt_n,
                          "one_core": {"value": k1 / dt_1, "rows": k1, "wall_s": dt_1}}

    # (i) the recipe: one process per core, one partition each, started together
    R = ssp.csr_matrix((Rx, Rj, Rp), shape=(m, p))
    Rcsc = R.tocsc()  # the recipe's operand: components_.T (CSC), converted by scipy per call
    del R
    nparts = max(1, min(cores, n // part))
    _G.update(ap=ap, aj=aj, ax=ax, m=m, part=part, Rcsc=Rcsc)
    ctx = mp.get_context("fork")
    _G["barrier"] = ctx.Barrier(nparts, timeout=600)
    t0 = time.perf_counter()
    with ctx.Pool(nparts) as pool:
        times = pool.map(_recipe_worker, range(nparts), chunksize=1)
    wall = time.perf_counter() - t0
    # one core alone (no neighbours sharing memory bandwidth)
    _G["barrier"] = ctx.Barrier(1)
    one = _recipe_worker(0)
    res["recipe"] = {"value": nparts * part / max(times), "processes": nparts, "part_rows": part,
                     "per_process_s": [round(t, 3) for t in times], "pool_wall_s": wall,
                     "one_core": {"value": part / one, "rows": part, "wall_s": one}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
