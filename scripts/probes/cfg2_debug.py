"""Debug probe: KDD-shaped launch of N rows with int64/int32 indptr, whole-output column check and
the location of the first bad entry (row, chunk, tile)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from randomprojection_amd import Projector, srp_matrix as sm, synth  # noqa: E402
from randomprojection_amd import _native as nat  # noqa: E402

n = int(sys.argv[1])
ipt = torch.int64 if sys.argv[2] == "i64" else torch.int32
staging = sys.argv[3]
R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
P = Projector(R)
P.set_staging(staging)
Ap, Aj, Ax = synth.kdd_rows_device(n, sm.KDD_M, seed=2021, indptr_dtype=ipt)
nnz_a = Aj.numel()
print("plan", P.plan(n, nnz_a), "nnz_a", nnz_a, flush=True)
ws = torch.empty(P.workspace_bytes(n, nnz_a), dtype=torch.uint8, device="cuda")
cap = int(1.02 * nnz_a * P.nnz / P.m) + 65536
Cp = torch.empty(n + 1, dtype=torch.int64 if cap >= 2**31 else torch.int32, device="cuda")
Cj = torch.full((cap,), -7, dtype=torch.int32, device="cuda")
Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
t0 = time.time()
nnz = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, workspace=ws, nnz_a=nnz_a)
print("nnz", nnz, "t", time.time() - t0, flush=True)
cp = Cp.to(torch.int64)
print("cp0", int(cp[0]), "cpN", int(cp[-1]), flush=True)
step = 1 << 28
for s in range(0, nnz, step):
    c = Cj[s:min(nnz, s + step)]
    bad = (c < 0) | (c >= 4096)
    if bool(bad.any()):
        i = s + int(torch.nonzero(bad)[0].item())
        nb = int(bad.sum().item())
        row = int(torch.searchsorted(cp, torch.tensor([i], device="cuda"), right=True).item()) - 1
        print(f"BAD entry {i} val {int(Cj[i])} row {row} chunk {row >> 27} tile {row // 256} bad_in_block {nb}",
              flush=True)
        lo = max(0, row - 3)
        print("cp around", cp[lo:row + 4].tolist(), flush=True)
        print("ap around", Ap[lo:row + 4].tolist(), flush=True)
        break
else:
    print("all columns ok", flush=True)
