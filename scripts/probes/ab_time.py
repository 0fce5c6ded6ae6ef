"""A/B timing of librp builds: configs[1] rows (uniform or power-law), one rp_project_device per
step, wall clock over K steps after W warmups (bench.py's step).
    python scripts/probes/ab_time.py [uniform|powerlaw] [path/to/librp_variant.so]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from randomprojection_amd import Projector, _native as nat, srp_matrix as sm, synth  # noqa: E402

dist = sys.argv[1] if len(sys.argv) > 1 else "uniform"
LIB = sys.argv[2] if len(sys.argv) > 2 else None
nat.load(LIB)
R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
P = Projector(R)
n = 119_705_032
Ap, Aj, Ax = synth.kdd_rows_device(n, sm.KDD_M, seed=2012, dist=dist)
nnz = Aj.numel()
ws = torch.empty(P.workspace_bytes(n, nnz), dtype=torch.uint8, device="cuda")
cap = int(1.05 * nnz * P.nnz / P.m) + 65536
Cp = torch.empty(n + 1, dtype=torch.int32, device="cuda")
Cj = torch.empty(cap, dtype=torch.int32, device="cuda")
Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, stream=st, workspace=ws, nnz_a=nnz)
for _ in range(3):
    P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, stream=st, workspace=ws, nnz_a=nnz, sync=False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, stream=st, workspace=ws, nnz_a=nnz, sync=False)
torch.cuda.synchronize()
print(LIB or "librp.so", nat.build_id(), dist, "ms/step", round((time.perf_counter() - t0) / 10 * 1e3, 3), "nnz", k,
      flush=True)
