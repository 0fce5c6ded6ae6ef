"""H2D / D2H copy rates on the box: pageable vs pinned, one stream (host boundary planning)."""
import json, time, sys
import numpy as np
import torch

torch.cuda.set_device(0)
nb = 384 << 20
host = np.ones(nb // 4, dtype=np.float32)
dev = torch.empty(nb // 4, dtype=torch.float32, device="cuda")
res = {}
def t(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps
ht = torch.from_numpy(host)
res["h2d_pageable_GBps"] = nb / t(lambda: dev.copy_(ht)) / 1e9
res["d2h_pageable_GBps"] = nb / t(lambda: ht.copy_(dev)) / 1e9
pin = torch.empty(nb // 4, dtype=torch.float32).pin_memory()
res["h2d_pinned_GBps"] = nb / t(lambda: dev.copy_(pin, non_blocking=True)) / 1e9
res["d2h_pinned_GBps"] = nb / t(lambda: pin.copy_(dev, non_blocking=True)) / 1e9
res["memcpy_1thread_GBps"] = nb / t(lambda: pin.numpy().__setitem__(slice(None), host)) / 1e9
torch.set_num_threads(16)
res["torch_copy_16threads_GBps"] = nb / t(lambda: pin.copy_(ht)) / 1e9
s2 = torch.cuda.Stream()
dev2 = torch.empty_like(dev); pin2 = torch.empty_like(pin).pin_memory()
def both():
    dev.copy_(pin, non_blocking=True)
    with torch.cuda.stream(s2):
        pin2.copy_(dev2, non_blocking=True)
    torch.cuda.current_stream().wait_stream(s2)
res["bidir_pinned_GBps_each"] = nb / t(both) / 1e9
print(json.dumps(res))
