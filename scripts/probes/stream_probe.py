"""Boundary-2 probe: configs[1]-shaped rows (uniform or power-law columns) streamed host CSR -> host
CSR through rp_project_stream; prints ms per pass, rp_project_stream_stats and the chunk count.
    python scripts/probes/stream_probe.py [uniform|powerlaw] [rows] [chunk_rows]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from randomprojection_amd import Projector, hostmem, srp_matrix as sm, synth  # noqa: E402

dist = sys.argv[1] if len(sys.argv) > 1 else "powerlaw"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 119_705_032
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 0
R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
P = Projector(R)
Ap, Aj, Ax = synth.kdd_rows_device(n, sm.KDD_M, seed=2013 if dist == "powerlaw" else 2012, dist=dist)
ap, aj, ax = Ap.cpu().numpy(), Aj.cpu().numpy(), Ax.cpu().numpy()
del Ap, Aj, Ax
torch.cuda.empty_cache()
nnz = aj.size
exp = nnz * P.nnz / P.m
cap = int(1.3 * exp) + 65536
out = (hostmem.empty(n + 1, np.int32), hostmem.empty(cap, np.int32), hostmem.empty(cap, np.float32))
for a in out:
    a.fill(0)
for it in range(4):
    t0 = time.perf_counter()
    cp, cj, cx = P.project_stream(ap, aj, ax, chunk_rows=chunk, out=out)
    dt = time.perf_counter() - t0
    print(dist, n, "chunk", chunk, "pass", it, f"{dt * 1e3:.1f} ms", f"{n / dt / 1e6:.1f} M rows/s", "nnz", cj.size,
          P.stream_stats(), flush=True)
