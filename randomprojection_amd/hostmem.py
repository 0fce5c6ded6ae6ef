"""Recycled host memory for results copied out of the GPU.

A fresh numpy array (``np.empty``) is an untouched anonymous mapping: the device-to-host copy
faults every page in, and in a process with the HIP runtime loaded those faults cost ~75 ms per GB
and do not parallelise (measured on the MI355X box, scripts/probes/d2h_probe.py and
d2h_thp_probe.py: 96 MB fresh 9.7 ms vs 1.8 ms into touched memory; 8 threads or
MADV_HUGEPAGE change nothing). For a 4M-row KDD2012 partition that is 16 of the ~28 ms of
``Projector.matmul``.

``empty(n, dtype)`` hands out ordinary numpy arrays whose memory comes from a pool of mappings
that were already faulted in. The array's base is a small holder object; when the last view of
the array dies, the holder's finaliser returns the mapping to the pool (bounded by
``RP_HOST_POOL_BYTES``, default 4 GiB of idle memory, past which mappings are unmapped). Arrays
the caller keeps are never touched again, so a result stays valid for as long as it is referenced.
"""
from __future__ import annotations

import collections
import mmap
import os
import threading
import weakref

import numpy as np

__all__ = ["empty", "pool_stats", "device_numa_node", "bind_to_device_numa"]

_MIN_POOLED = 1 << 20          # smaller requests: np.empty (malloc's own heap reuses them)
_GRAIN = 2 << 20               # mapping sizes are multiples of 2 MiB
_lock = threading.Lock()
_free: dict[int, list] = collections.defaultdict(list)   # size -> idle mappings
_returned: collections.deque = collections.deque()       # filled by finalisers (any thread, no lock)
_idle_bytes = 0
_stats = {"hits": 0, "misses": 0, "unmapped": 0}


def _limit() -> int:
    return int(os.environ.get("RP_HOST_POOL_BYTES", 4 << 30))


class _Holder:
    """Base object of a pooled array (exposes the mapping through ``__array_interface__``)."""

    __slots__ = ("__array_interface__", "mm", "__weakref__")


def _drain_locked() -> None:
    global _idle_bytes
    while _returned:
        mm = _returned.popleft()
        _free[len(mm)].append(mm)
        _idle_bytes += len(mm)
    limit = _limit()
    while _idle_bytes > limit and _free:
        size = max(_free)            # drop the largest idle mappings first
        mm = _free[size].pop()
        if not _free[size]:
            del _free[size]
        _idle_bytes -= size
        _stats["unmapped"] += 1
        mm.close()


def _take(nbytes: int):
    global _idle_bytes
    size = max(_GRAIN, (nbytes + _GRAIN - 1) // _GRAIN * _GRAIN)
    with _lock:
        _drain_locked()
        # best fit among idle mappings no larger than 2x the request
        fits = [s for s in _free if size <= s <= 2 * size]
        if fits:
            s = min(fits)
            mm = _free[s].pop()
            if not _free[s]:
                del _free[s]
            _idle_bytes -= s
            _stats["hits"] += 1
            return mm
        _stats["misses"] += 1
    return mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)


def empty(n: int, dtype) -> np.ndarray:
    """``np.empty(n, dtype)`` backed by recycled, already-faulted memory (1-D, C-contiguous)."""
    dtype = np.dtype(dtype)
    nbytes = int(n) * dtype.itemsize
    if nbytes < _MIN_POOLED:
        return np.empty(n, dtype)
    mm = _take(nbytes)
    addr = np.frombuffer(mm, np.uint8, 1).ctypes.data   # the mapping's address (view dropped below)
    h = _Holder()
    h.mm = mm
    h.__array_interface__ = {"data": (addr, False), "shape": (int(n),), "typestr": dtype.str, "version": 3}
    weakref.finalize(h, _returned.append, mm)
    return np.asarray(h)


def pool_stats() -> dict:
    with _lock:
        _drain_locked()
        return dict(_stats, idle_bytes=_idle_bytes, idle_mappings=sum(len(v) for v in _free.values()))


def device_numa_node(device: int):
    """NUMA node of a GPU's PCIe attachment (sysfs), or None when it cannot be determined."""
    try:
        import torch

        pr = torch.cuda.get_device_properties(device)
        bus, dev = getattr(pr, "pci_bus_id", None), getattr(pr, "pci_device_id", None)
        if bus is None or dev is None:
            return None
        dom = int(getattr(pr, "pci_domain_id", 0) or 0)
        with open(f"/sys/bus/pci/devices/{dom:04x}:{int(bus):02x}:{int(dev):02x}.0/numa_node") as f:
            node = int(f.read().strip())
        return node if node >= 0 else None
    except Exception:  # noqa: BLE001 - sysfs layouts vary; binding is an optimisation only
        return None


def _cpulist(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def bind_to_device_numa(device: int) -> dict:
    """Restrict this process to the CPUs of its GPU's NUMA node (when the node is known and shares
    CPUs with the current affinity), so host buffers it allocates and first-touches afterwards
    (pinned staging, result arrays) sit next to the GPU's PCIe root: with 8 ranks streaming host
    CSR at once, every rank then draws on its own socket's DRAM channels. Returns what was done."""
    node = device_numa_node(device)
    if node is None:
        return {"numa_node": None, "bound_cpus": None}
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            want = _cpulist(f.read())
        have = os.sched_getaffinity(0)
        cpus = want & have
        if not cpus:
            return {"numa_node": node, "bound_cpus": None}
        os.sched_setaffinity(0, cpus)
        return {"numa_node": node, "bound_cpus": len(cpus)}
    except OSError:
        return {"numa_node": node, "bound_cpus": None}
