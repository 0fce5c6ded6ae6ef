import os, sys, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ["RP_PIPE"] = "lpr"
from randomprojection_amd import Projector, srp_matrix as sm, synth
m, p = sm.KDD_M, 4096
R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
P = Projector(R)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
Ap, Aj, Ax = synth.kdd_rows_device(n, m, seed=5)
def run(stage):
    P.set_staging(stage)
    nnz = Aj.numel()
    ws = torch.empty(P.workspace_bytes(n, nnz), dtype=torch.uint8, device="cuda")
    cap = int(1.05 * nnz * P.nnz / P.m) + 65536
    Cp = torch.empty(n + 1, dtype=torch.int32, device="cuda"); Cj = torch.empty(cap, dtype=torch.int32, device="cuda"); Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
    k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, workspace=ws, nnz_a=nnz)
    return Cp.cpu().numpy(), Cj[:k].cpu().numpy(), Cx[:k].cpu().numpy()
a = run("off"); b = run("on")
print("nnz", a[1].size, b[1].size)
d = np.nonzero(a[0] != b[0])[0]
print("first indptr diff rows", d[:10], "count", d.size)
if d.size:
    r = d[0] - 1 if d[0] > 0 else 0
    for rr in range(max(0, r - 1), r + 3):
        print(rr, a[1][a[0][rr]:a[0][rr+1]], b[1][b[0][rr]:b[0][rr+1]])
        print("  A cols", Aj[Ap[rr]:Ap[rr+1]].cpu().numpy())
