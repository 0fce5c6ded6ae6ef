"""Fresh-destination D2H: is the cost page faults or HIP's per-call pinning of new pageable memory?"""
import json, threading, time
import numpy as np
import torch
torch.cuda.set_device(0)
nb = 96 << 20
src = torch.ones(nb // 4, dtype=torch.float32, device="cuda")
res = {}
def touch(a, nt=8):
    v = a.view(np.uint8); per = (v.size // nt + 4095) & ~4095
    ts = [threading.Thread(target=lambda i=i: v[i * per:(i + 1) * per:4096].fill(0)) for i in range(nt)]
    [t.start() for t in ts]; [t.join() for t in ts]
def run(name, fn, reps=4):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter(); fn(); torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    res[name + "_ms"] = best * 1e3
def fresh():
    a = np.empty(nb // 4, np.float32); torch.from_numpy(a).copy_(src)
def fresh_prefault():
    a = np.empty(nb // 4, np.float32); touch(a); torch.from_numpy(a).copy_(src)
def fresh_prefault_only():
    a = np.empty(nb // 4, np.float32); touch(a)
keep = np.ones(nb // 4, np.float32)
def reused():
    torch.from_numpy(keep).copy_(src)
pin = torch.empty(nb // 4, dtype=torch.float32).pin_memory()
def via_pinned():
    pin.copy_(src, non_blocking=True); torch.cuda.synchronize()
    a = np.empty(nb // 4, np.float32)
    torch.set_num_threads(16); torch.from_numpy(a).copy_(pin)
run("fresh", fresh); run("fresh_prefault8", fresh_prefault); run("prefault8_only", fresh_prefault_only)
run("reused", reused); run("via_pinned_then_16thread_copy", via_pinned)
res["MB"] = nb >> 20
print(json.dumps(res))
