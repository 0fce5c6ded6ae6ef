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

__all__ = ["empty", "pool_stats"]

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
