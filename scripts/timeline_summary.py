"""Summarise a rocprofv3 kernel + memory-copy trace (csv): over the last timed window, busy time of
kernels and of each copy direction, their overlap, and the idle gaps. Usage: timeline_summary.py DIR"""
import csv
import glob
import sys


def load(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            out.append(r)
    return out


def union(iv):
    iv = sorted(iv)
    res = []
    for s, e in iv:
        if res and s <= res[-1][1]:
            res[-1][1] = max(res[-1][1], e)
        else:
            res.append([s, e])
    return res


def total(iv):
    return sum(e - s for s, e in iv)


def inter(a, b):
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


d = sys.argv[1]
ks = load(d + "/**/*kernel_trace.csv")
ms = load(d + "/**/*memory_copy_trace.csv")
kiv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ks]
# window: from the last 'line_count_kernel' minus the span of one step... use the last 40% of the trace
t0 = min(s for s, _, _ in kiv)
t1 = max(e for _, e, _ in kiv)
w0 = t0 + int(0.6 * (t1 - t0))
K = union([(max(s, w0), e) for s, e, _ in kiv if e > w0])
by = {}
for r in ms:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= w0:
        continue
    by.setdefault(r.get("Direction", r.get("Kind", "?")), []).append((max(s, w0), e))
print(f"window {(t1 - w0) / 1e6:.1f} ms: kernels busy {total(K) / 1e6:.1f} ms")
for k, v in by.items():
    u = union(v)
    print(f"  copies {k}: n={len(v)} busy {total(u) / 1e6:.1f} ms, overlapping kernels {inter(u, K) / 1e6:.1f} ms, "
          f"bytes {sum(int(r.get('Size', 0)) for r in ms if int(r['End_Timestamp']) > w0 and r.get('Direction', r.get('Kind', '?')) == k) / 1e9:.2f} GB")
names = {}
for s, e, n in kiv:
    if e > w0:
        names[n[:40]] = names.get(n[:40], 0) + (e - max(s, w0))
for n, t in sorted(names.items(), key=lambda x: -x[1])[:8]:
    print(f"  {n:40s} {t / 1e6:8.2f} ms")
