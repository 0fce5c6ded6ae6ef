"""In a GPU process: fresh host arrays with and without madvise(MADV_HUGEPAGE) before the first touch."""
import ctypes, json, time
import numpy as np
import torch
torch.cuda.set_device(0)
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
nb = 96 << 20
src = torch.ones(nb // 4, dtype=torch.float32, device="cuda")
res = {}
def huge(a):
    base = a.ctypes.data; lo = (base + (2 << 20) - 1) & ~((2 << 20) - 1)
    n = (base + a.nbytes - lo) & ~((2 << 20) - 1)
    return libc.madvise(lo, n, 14)
def run(name, fn, reps=4):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter(); fn(); torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    res[name + "_ms"] = best * 1e3
run("touch_4k", lambda: np.empty(nb // 4, np.float32).view(np.uint8)[::4096].fill(0))
def th():
    a = np.empty(nb // 4, np.float32); huge(a); a.view(np.uint8)[::4096].fill(0)
run("touch_huge", th)
run("d2h_fresh_4k", lambda: torch.from_numpy(np.empty(nb // 4, np.float32)).copy_(src))
def dh():
    a = np.empty(nb // 4, np.float32); huge(a); torch.from_numpy(a).copy_(src)
run("d2h_fresh_huge", dh)
a = np.empty(nb // 4, np.float32); res["madvise_rc"] = huge(a)
print(json.dumps(res))
