"""Page-fault cost of fresh host output arrays: 4 KB faults vs madvise(MADV_HUGEPAGE), 1 vs N threads."""
import ctypes, json, mmap, os, threading, time
import numpy as np
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
res = {}
for f in ("enabled", "defrag"):
    try:
        res["thp_" + f] = open(f"/sys/kernel/mm/transparent_hugepage/{f}").read().strip()
    except OSError as e:
        res["thp_" + f] = str(e)
nb = 200 << 20
def touch(a, nt):
    v = a.view(np.uint8)
    per = (v.size // nt + 4095) & ~4095
    def w(i):
        v[i * per:(i + 1) * per:4096] = 1
    ts = [threading.Thread(target=w, args=(i,)) for i in range(nt)]
    [t.start() for t in ts]; [t.join() for t in ts]
for adv in (False, True):
    for nt in (1, 8, 16):
        best = 1e9
        for _ in range(3):
            a = np.empty(nb, np.uint8)
            if adv:
                base = a.ctypes.data; lo = (base + (2 << 20) - 1) & ~((2 << 20) - 1)
                libc.madvise(lo, (base + nb - lo) & ~((2 << 20) - 1), 14)
            t0 = time.perf_counter(); touch(a, nt); best = min(best, time.perf_counter() - t0)
            del a
        res[f"touch_{'huge' if adv else '4k'}_{nt}t_GBps"] = nb / best / 1e9
print(json.dumps(res))
