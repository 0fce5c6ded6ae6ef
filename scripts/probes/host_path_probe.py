"""(Historical, round 1: it sets environment knobs librp no longer reads — rp_projector_set_option
replaced them in round 3; kept as the record of DESIGN.md §3d's measurement.)
Where does the host CSR -> host CSR call (boundary 2) spend its time? Components timed separately."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch
torch.cuda.set_device(0)
from randomprojection_amd import Projector, srp_matrix as sm
from bench_host import kdd_csr

def tm(fn, reps=3):
    fn(); torch.cuda.synchronize(); best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t0)
    return best * 1e3

R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
P = Projector(R)
A = kdd_csr(np.random.default_rng(2012), 4_000_000, sm.KDD_M)
res = {"rows": A.shape[0], "nnz_a": int(A.nnz)}
res["matmul_ms"] = tm(lambda: P.matmul(A))
for th in ("0", "4", "16"):
    os.environ["RP_HOST_THREADS"] = th
    res[f"matmul_ms_threads{th}"] = tm(lambda: P.matmul(A), reps=5)
os.environ.pop("RP_HOST_THREADS")
C = P.matmul(A)
res["nnz_c"] = int(C.nnz)
dev = {}
def h2d():
    dev["p"] = torch.from_numpy(A.indptr).cuda(); dev["j"] = torch.from_numpy(A.indices).cuda(); dev["x"] = torch.from_numpy(A.data).cuda()
res["h2d_torch_ms"] = tm(h2d)
Cp = torch.empty(A.shape[0] + 1, dtype=torch.int32, device="cuda")
cap = int(C.nnz * 1.1)
Cj = torch.empty(cap, dtype=torch.int32, device="cuda"); Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
res["device_project_ms"] = tm(lambda: P.project_device(dev["p"], dev["j"], dev["x"], Cp, Cj, Cx, nnz_a=A.nnz))
k = C.nnz
def d2h_fresh():
    a = np.empty(A.shape[0] + 1, np.int32); b = np.empty(k, np.int32); c = np.empty(k, np.float32)
    torch.from_numpy(a).copy_(Cp); torch.from_numpy(b).copy_(Cj[:k]); torch.from_numpy(c).copy_(Cx[:k])
res["d2h_fresh_ms"] = tm(d2h_fresh)
a = np.ones(A.shape[0] + 1, np.int32); b = np.ones(k, np.int32); c = np.ones(k, np.float32)
def d2h_warm():
    torch.from_numpy(a).copy_(Cp); torch.from_numpy(b).copy_(Cj[:k]); torch.from_numpy(c).copy_(Cx[:k])
res["d2h_prefaulted_ms"] = tm(d2h_warm)
res["np_empty_touch_ms"] = tm(lambda: (np.empty(k, np.int32).fill(1), np.empty(k, np.float32).fill(1)))
def mono():
    ip = A.indptr
    return bool(np.all(ip[1:] >= ip[:-1]))
res["host_monotone_check_numpy_ms"] = tm(mono)
print(json.dumps(res))
