"""Debug probe: a window of rows of the 500M-row synthetic matrix (seed 2021) run alone, staged vs
direct row-lane, whole outputs compared; prints the differing rows' outputs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from randomprojection_amd import Projector, srp_matrix as sm, synth  # noqa: E402

N, r0, nr = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
Ap, Aj, Ax = synth.kdd_rows_device(N, sm.KDD_M, seed=2021, indptr_dtype=torch.int64)
e0, e1 = int(Ap[r0]), int(Ap[r0 + nr])
ap = (Ap[r0:r0 + nr + 1] - e0).to(torch.int32).contiguous()
aj = Aj[e0:e1].clone()
ax = Ax[e0:e1].clone()
del Ap, Aj, Ax
torch.cuda.empty_cache()
print("window entries", e1 - e0, "first entry", e0, flush=True)
outs = {}
for st in ("off", "on"):
    P = Projector(R)
    P.set_staging(st)
    n, nnz_a = nr, e1 - e0
    ws = torch.empty(P.workspace_bytes(n, nnz_a), dtype=torch.uint8, device="cuda")
    cap = int(1.05 * nnz_a * 0.554) + 65536
    Cp = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    Cj = torch.empty(cap, dtype=torch.int32, device="cuda")
    Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
    nnz = P.project_device(ap, aj, ax, Cp, Cj, Cx, workspace=ws, nnz_a=nnz_a)
    print(st, P.plan(n, nnz_a), nnz, "deferred/heavy", int(ws[16:20].view(torch.int32).item()), flush=True)
    outs[st] = (Cp, Cj[:nnz], Cx[:nnz])
    P.close()
a, b = outs["off"], outs["on"]
d = torch.nonzero(a[0] != b[0]).flatten()
print("indptr differs at", d.numel(), d[:10].tolist(), flush=True)
if d.numel():
    r = int(d[0]) - 1
    for name, o in (("off", a), ("on", b)):
        print(name, "row", r, o[1][int(o[0][r]):int(o[0][r + 1])].tolist(), flush=True)
    t = r // 256
    print("tile", t, "rows of tile: entries", int(ap[min(nr, t * 256 + 256)] - ap[t * 256]), flush=True)
