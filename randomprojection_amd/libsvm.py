"""libsvm ingest on the GPU.

Replaces ``spark.read.format("libsvm").load(path, numFeatures=N_FEATURES)`` +
``.withColumn("id", f.monotonically_increasing_id())`` (code/clustermode/randomProjection.py:71-72,
code/localmode/randomProjection.py:92-96): text is read in newline-aligned chunks (a chunk plays
the role of a Spark partition), copied to HBM and parsed by librp's ``rp_libsvm_parse_device``
kernels into CSR (0-based ascending int32 indices, float32 values, float64 labels). Row ids follow
``monotonically_increasing_id``: ``(chunk_index << 33) + row_in_chunk``.

``project_libsvm`` chains ingest and projection on the device (boundary 3 of SURVEY.md §8(d):
libsvm text -> projected CSR), so A never round-trips through the host.
"""
from __future__ import annotations

import ctypes
import mmap
import os

import numpy as np
import scipy.sparse as sp

from . import _native as nat
from . import hostmem

__all__ = ["parse_device", "parse_bytes", "iter_chunks", "split_range", "load_libsvm", "project_libsvm",
           "project_text_stream", "libsvm_to_parquet", "partition_ids"]

DEFAULT_CHUNK = 256 << 20


class LibsvmFormatError(ValueError):
    def __init__(self, msg, line):
        super().__init__(msg)
        self.line = line


def partition_ids(chunk_index: int, n_rows: int) -> np.ndarray:
    """Spark ``monotonically_increasing_id``: partition id in the upper 31 bits, row in the lower 33."""
    return (np.int64(chunk_index) << np.int64(33)) + np.arange(n_rows, dtype=np.int64)


def parse_device(text, n_bytes: int, num_features: int, device: int = 0, stream=None, indptr_dtype=None):
    """Parse libsvm text already in device memory (a uint8 torch tensor, 16-byte aligned).
    Returns torch tensors (labels f64, indptr, indices i32, data f32) on ``cuda:device``. The kernels
    run on ``stream`` (default: torch's current stream of that device, the stream the tensors are
    allocated and filled on, so the caching allocator's reuse stays ordered)."""
    import torch

    lib = nat.load()
    dev = torch.device("cuda", device)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    rows, nnz, err = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(-1)
    tp = ctypes.c_void_p(text.data_ptr())
    nat.check(lib.rp_libsvm_parse_device(device, tp, n_bytes, num_features, None, None, nat.RP_I64, None, None,
                                         0, 0, ctypes.c_void_p(stream), ctypes.byref(rows), ctypes.byref(nnz),
                                         ctypes.byref(err)))
    n, k = int(rows.value), int(nnz.value)
    if indptr_dtype is None:
        indptr_dtype = torch.int32 if k < 2**31 else torch.int64
    labels = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    indptr = torch.empty(n + 1, dtype=indptr_dtype, device=dev)
    indices = torch.empty(max(k, 1), dtype=torch.int32, device=dev)
    data = torch.empty(max(k, 1), dtype=torch.float32, device=dev)
    rc = lib.rp_libsvm_parse_device(device, tp, n_bytes, num_features, ctypes.c_void_p(labels.data_ptr()),
                                    ctypes.c_void_p(indptr.data_ptr()),
                                    nat.RP_I64 if indptr_dtype == torch.int64 else nat.RP_I32,
                                    ctypes.c_void_p(indices.data_ptr()), ctypes.c_void_p(data.data_ptr()), n, k,
                                    ctypes.c_void_p(stream), ctypes.byref(rows), ctypes.byref(nnz), ctypes.byref(err))
    if rc == nat.RP_ERR_INVALID and err.value >= 0:
        raise LibsvmFormatError(lib.rp_last_error().decode(), int(err.value))
    nat.check(rc)
    return labels[:n], indptr, indices[:k], data[:k]


def _to_device(buf, device):
    """Copy a bytes-like chunk (bytes, bytearray, or a memoryview of the mapped file) to a 16-byte
    aligned device buffer with one host->device copy and no host-side copy."""
    import warnings

    import torch

    n = len(buf)
    t = torch.empty((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=torch.device("cuda", device))
    if n:
        with warnings.catch_warnings():  # read-only source (mapped file): torch only reads it
            warnings.simplefilter("ignore", UserWarning)
            src = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8, count=n))
        t[:n].copy_(src)
    return t, n


def parse_bytes(buf, num_features: int, device: int = 0):
    """Parse a bytes-like chunk of libsvm text -> (labels float64, scipy CSR float32)."""
    t, n = _to_device(buf, device)
    labels, indptr, indices, data = parse_device(t, n, num_features, device)
    X = sp.csr_matrix((data.cpu().numpy(), indices.cpu().numpy(), indptr.cpu().numpy()),
                      shape=(int(labels.numel()), num_features))
    return labels.cpu().numpy(), X


def split_range(mm, size: int, lo: int, hi: int):
    """The byte range of the lines that START in [lo, hi) (Hadoop's line-record split rule, which
    Spark's text sources follow): a line straddling ``lo`` belongs to the previous split, the line
    straddling ``hi`` to this one. Splits of consecutive ranges cover every line exactly once."""
    lo, hi = max(0, min(lo, size)), max(0, min(hi, size))

    def line_start_at_or_after(b):
        if b <= 0:
            return 0
        if b >= size:
            return size
        if mm[b - 1:b] == b"\n":
            return b
        nl = mm.find(b"\n", b)
        return size if nl < 0 else nl + 1

    return line_start_at_or_after(lo), line_start_at_or_after(hi)


def iter_chunks(path: str, chunk_bytes: int = DEFAULT_CHUNK, copy: bool = True, byte_range=None):
    """Newline-aligned chunks of a file (memory-mapped, never loaded whole). ``copy=False`` yields
    memoryviews of the mapping instead of bytes: each is valid until the next chunk is requested
    and must be released (``del``) by then. ``byte_range=(lo, hi)``: only the lines that start in
    [lo, hi) (one rank's split of the file, see ``split_range``)."""
    size = os.path.getsize(path)
    if size == 0:
        return
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as mm:
        start, stop = (0, size) if byte_range is None else split_range(mm, size, *byte_range)
        size = stop
        while start < size:
            end = min(start + chunk_bytes, size)
            if end < size:
                nl = mm.rfind(b"\n", start, end)
                if nl >= 0:
                    end = nl + 1
                else:  # one line longer than a chunk: extend to its end
                    nxt = mm.find(b"\n", end)
                    end = size if nxt < 0 else nxt + 1
            view = memoryview(mm)[start:end]
            if copy:
                chunk = view.tobytes()
                view.release()
                yield chunk
            else:
                yield view
                view.release()
            start = end


def load_libsvm(path: str, num_features: int, chunk_bytes: int = DEFAULT_CHUNK, device: int = 0):
    """Yield ``(ids, labels, X)`` per chunk — the rows of one Spark partition each."""
    for ci, buf in enumerate(iter_chunks(path, chunk_bytes)):
        labels, X = parse_bytes(buf, num_features, device)
        yield partition_ids(ci, X.shape[0]), labels, X


def project_libsvm(path: str, projector, chunk_bytes: int = DEFAULT_CHUNK, order: str = "sorted",
                   byte_range=None, partition_base: int = 0):
    """libsvm text -> GPU parse -> GPU projection -> host CSR, per chunk: yields
    ``(ids, labels, C)`` with ``C`` = the chunk's rows of ``X @ R`` (scipy CSR, float32).
    ``byte_range``: only the lines starting in [lo, hi) (a rank's split); chunk k gets partition id
    ``partition_base + k`` in its row ids."""
    import torch

    dev = projector.device
    st = torch.cuda.current_stream(torch.device("cuda", dev)).cuda_stream  # where torch fills/frees the tensors
    for ci, buf in enumerate(iter_chunks(path, chunk_bytes, copy=False, byte_range=byte_range)):
        t, n = _to_device(buf, dev)
        del buf  # the view must be gone before the next chunk (the mapping closes at the end)
        labels, Ap, Aj, Ax = parse_device(t, n, projector.m, dev, stream=st)
        del t
        rows = int(labels.numel())
        cap = int(1.3 * Aj.numel() * projector.nnz / max(projector.m, 1)) + 1024
        Cp = torch.empty(rows + 1, dtype=torch.int64, device=torch.device("cuda", dev))
        Cj = torch.empty(cap, dtype=torch.int32, device=Cp.device)
        Cx = torch.empty(cap, dtype=torch.float32, device=Cp.device)
        try:
            k = projector.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=order, nnz_a=int(Aj.numel()), stream=st)
        except nat.RPError as e:
            if e.code != nat.RP_ERR_CAPACITY:
                raise
            Cj = torch.empty(e.nnz, dtype=torch.int32, device=Cp.device)
            Cx = torch.empty(e.nnz, dtype=torch.float32, device=Cp.device)
            k = projector.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=order, nnz_a=int(Aj.numel()), stream=st)
        if k < 2**31:  # the index dtype scipy's csr_matrix settles on
            Cp = Cp.to(torch.int32)
        C = sp.csr_matrix((_download(Cx[:k]), _download(Cj[:k]), _download(Cp)), shape=(rows, projector.p))
        yield partition_ids(partition_base + ci, rows), _download(labels), C


def project_text_stream(text, projector, order: str = "sorted", chunk_bytes: int = 64 << 20, out=None,
                        out_index_dtype=None):
    """Boundary 3 in one native call (rp_libsvm_project_stream): libsvm text in host memory (a uint8
    numpy array, bytes or a mapped file's memoryview) -> chunks of whole lines uploaded, parsed and
    projected on the GPU with upload, compute and download overlapped -> host arrays
    ``(labels f64, indptr, indices, data f32)`` of ``X @ R`` for every row of the text.

    ``out``: optional preallocated ``(labels, indptr, indices, data)`` host arrays (pinned or
    pageable; capacities = their lengths) -- the steady-state form, nothing allocated per call.
    Without it the capacities come from counting newlines and ':' in the text, with one exact retry."""
    a = np.frombuffer(text, dtype=np.uint8) if not isinstance(text, np.ndarray) else text.reshape(-1).view(np.uint8)
    lib = nat.load()
    odx = {"sorted": nat.RP_ORDER_SORTED, "scipy": nat.RP_ORDER_SCIPY}[order]
    if out is None:
        rows_cap = int(np.count_nonzero(a == 10)) + 1
        items = int(np.count_nonzero(a == 58))
        exp = items * projector.nnz / max(projector.m, 1)
        cap = int(1.05 * exp + 8 * np.sqrt(exp + 1)) + 65536
    else:
        # the native side trusts these sizes: check them against each other before the call
        labels, ip, ix, dx = out
        for name, arr, want in (("labels", labels, (np.float64,)), ("indptr", ip, (np.int32, np.int64)),
                                ("indices", ix, (np.int32, np.int64)), ("data", dx, (np.float32,))):
            if not isinstance(arr, np.ndarray) or arr.ndim != 1 or arr.dtype not in [np.dtype(w) for w in want] \
                    or not arr.flags.c_contiguous or not arr.flags.writeable:
                raise TypeError(f"out {name}: a writeable contiguous 1-D array of {[np.dtype(w).name for w in want]}")
        if ix.size != dx.size:
            raise ValueError(f"out indices ({ix.size}) and data ({dx.size}) must have the same length")
        if ip.size < labels.size + 1:
            raise ValueError(f"out indptr needs labels.size + 1 = {labels.size + 1} entries, has {ip.size}")
        rows_cap, cap = labels.size, dx.size
    for _ in range(2):
        if out is None:
            it = np.dtype(out_index_dtype or (np.int32 if cap < 2**31 else np.int64))
            o = (np.empty(rows_cap, np.float64), np.empty(rows_cap + 1, it), np.empty(max(cap, 1), it),
                 np.empty(max(cap, 1), np.float32))
        else:
            o = out
        labels, ip, ix, dx = o
        co = nat.CsrOut(ip.ctypes.data, nat.idx_code(ip.dtype), ix.ctypes.data, nat.idx_code(ix.dtype),
                        dx.ctypes.data, int(dx.size if cap > 0 else 0))
        n, k, el = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(-1)
        rc = lib.rp_libsvm_project_stream(projector._h, ctypes.c_void_p(a.ctypes.data), int(a.size), odx,
                                          int(chunk_bytes), ctypes.c_void_p(labels.ctypes.data), int(labels.size),
                                          ctypes.byref(co), ctypes.byref(n), ctypes.byref(k), ctypes.byref(el))
        if rc == nat.RP_ERR_INVALID and el.value >= 0:
            raise LibsvmFormatError(lib.rp_last_error().decode(), int(el.value))
        if rc == nat.RP_ERR_CAPACITY and out is None and k.value > cap:
            cap = int(k.value)
            continue
        nat.check(rc)
        rows, nnz = int(n.value), int(k.value)
        return labels[:rows], ip[:rows + 1], ix[:nnz], dx[:nnz]
    raise RuntimeError("capacity retry failed")


def libsvm_to_parquet(path: str, projector, out_dir: str, chunk_bytes: int = DEFAULT_CHUNK, byte_range=None,
                      partition_base: int = 0, compression: str = "snappy"):
    """The recipe end to end for one rank: libsvm text -> GPU parse -> GPU projection -> one Parquet
    part file per chunk (``part-<partition>.parquet``, schema (id Long, label Float, features
    VectorUDT), code/clustermode/randomProjection.py:71-80,107-113). Returns the part file paths."""
    from . import egress

    os.makedirs(out_dir, exist_ok=True)
    parts = []
    for ids, labels, C in project_libsvm(path, projector, chunk_bytes, order="sorted", byte_range=byte_range,
                                         partition_base=partition_base):
        pid = int(ids[0] >> 33) if len(ids) else partition_base + len(parts)
        f = os.path.join(out_dir, f"part-{pid:08d}.parquet")
        egress.write_parquet(f, ids, labels, C, compression=compression)
        parts.append(f)
    return parts


def _download(t):
    """Device tensor -> host array in recycled, already-faulted memory (hostmem.py)."""
    import torch

    out = hostmem.empty(t.numel(), torch.empty(0, dtype=t.dtype).numpy().dtype)
    torch.from_numpy(out).copy_(t)
    return out
