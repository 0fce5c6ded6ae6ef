"""R resident on one MI355X and the product ``A @ R`` computed by librp's HIP kernel.

Replaces, in the reference (paths relative to /root/reference):
  * ``local_rnd_mat = srp.components_.T.astype(np.float32)``   code/clustermode/randomProjection.py:101
  * ``sc.broadcast(local_rnd_mat)``                              code/clustermode/randomProjection.py:104
  * ``features_matrix.dot(local_csr_matrix)``                    code/clustermode/randomProjection.py:46
    -> scipy ``_matmul_sparse`` (scipy/sparse/_compressed.py:546-604): ``other = self.__class__(other)``
       then ``csr_matmat_maxnnz`` + ``csr_matmat``.

``Projector.matmul(A)`` returns exactly what ``A @ R`` returns in scipy for CSR ``A``: same
container type, same value dtype (``upcast``), same index dtype rule (``get_index_dtype`` with
``check_contents=False``), same per-row storage order, same values bit for bit.
There is no CPU fallback: a missing library or GPU raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading
import weakref

import numpy as np
import scipy.sparse as sp

from . import _native as nat
from . import hostmem

__all__ = ["Projector", "get_projector", "scipy_result_index_dtype"]

_INT32_MAX = np.iinfo(np.int32).max
# host matrices from this many rows go through the chunked stream path (rp_project_stream)
STREAM_MIN_ROWS = 8 << 20


def _operand_csr(R) -> sp.csr_matrix:
    """scipy's ``other = self.__class__(other)`` (scipy/sparse/_compressed.py:564): a CSR view of a
    CSR input (storage order kept), ``csc_tocsr`` for CSC (rows sorted by column), ``tocsr`` else."""
    if sp.issparse(R):
        return R if (R.format == "csr" and isinstance(R, sp.csr_matrix)) else sp.csr_matrix(R)
    R = np.asarray(R)
    if R.ndim != 2:
        raise ValueError("R must be 2-D")
    return sp.csr_matrix(R)


def scipy_result_index_dtype(arrays, nnz) -> np.dtype:
    """``_get_index_dtype(arrays, maxval=nnz)`` of ``_matmul_sparse`` (check_contents=False)."""
    if nnz > _INT32_MAX:
        return np.dtype(np.int64)
    for a in arrays:
        if not np.can_cast(np.asarray(a).dtype, np.int32):
            return np.dtype(np.int64)
    return np.dtype(np.int32)


class Projector:
    """An m x p projection matrix R uploaded once to ``device`` (HBM resident).

    ``layout``: "auto" (packed single-magnitude layout when R qualifies — every
    SparseRandomProjection matrix does — else generic CSR), "packed" or "generic".
    """

    def __init__(self, R=None, device: int = 0, layout: str = "auto", *, _handle=None, _meta=None):
        self._lib = nat.load()
        self._lock = threading.Lock()
        self.device = int(device)
        if _handle is not None:
            self._h = _handle
            self.r_index_dtype, self.dtype = _meta
        else:
            Rc = _operand_csr(R)
            if Rc.dtype not in (np.float32, np.float64):
                Rc = Rc.astype(np.float64)
            self.r_index_dtype = np.result_type(Rc.indptr.dtype, Rc.indices.dtype)
            self.dtype = Rc.dtype
            code = {"auto": nat.RP_LAYOUT_AUTO, "generic": nat.RP_LAYOUT_GENERIC, "packed": nat.RP_LAYOUT_PACKED}[layout]
            indptr = np.ascontiguousarray(Rc.indptr)
            indices = np.ascontiguousarray(Rc.indices)
            data = np.ascontiguousarray(Rc.data)
            h = ctypes.c_void_p()
            nat.check(self._lib.rp_projector_create(
                self.device, Rc.shape[0], Rc.shape[1], nat.ptr(indptr), nat.idx_code(indptr.dtype),
                nat.ptr(indices), nat.idx_code(indices.dtype), nat.ptr(data), nat.val_code(data.dtype),
                code, ctypes.byref(h)))
            self._h = h
        info = nat.ProjectorInfo()
        nat.check(self._lib.rp_projector_info_get(self._h, ctypes.byref(info)))
        self.info = info
        self.m, self.p, self.nnz = int(info.m), int(info.p), int(info.nnz)
        self.layout = "packed" if info.layout == nat.RP_LAYOUT_PACKED else "generic"
        self.shape = (self.m, self.p)

    # -------------------------------------------------------------------------------- lifetime
    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.rp_projector_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------------------------- image
    def image_nbytes(self):
        return [int(self.info.buffer_bytes[i]) for i in range(self.info.n_buffers)]

    def export_image(self, dst_ptrs, stream=0):
        """Copy the device image into caller device buffers (e.g. torch tensors to broadcast)."""
        for i, dst in enumerate(dst_ptrs):
            nat.check(self._lib.rp_projector_export(self._h, i, ctypes.c_void_p(int(dst)), ctypes.c_void_p(stream)))

    @classmethod
    def from_image(cls, info: "nat.ProjectorInfo", src_ptrs, device: int, r_index_dtype=np.int32, dtype=np.float32):
        """Build a projector from an image already in device memory (after an RCCL broadcast)."""
        lib = nat.load()
        arr = (ctypes.c_void_p * len(src_ptrs))(*[ctypes.c_void_p(int(s)) for s in src_ptrs])
        h = ctypes.c_void_p()
        nat.check(lib.rp_projector_create_from_device(int(device), ctypes.byref(info), arr, ctypes.byref(h)))
        return cls(device=device, _handle=h, _meta=(np.dtype(r_index_dtype), np.dtype(dtype)))

    # -------------------------------------------------------------------------------- host path
    def compute_dtype(self, a_dtype) -> np.dtype:
        T = np.result_type(np.dtype(a_dtype), self.dtype)
        if T == np.float16:
            T = np.dtype(np.float32)
        if T not in (np.float32, np.float64):
            raise TypeError(f"unsupported value dtype {T} (float32/float64 only)")
        return np.dtype(T)

    def project_arrays(self, indptr, indices, data, n_cols=None, order: str = "scipy", out_index_dtype=None):
        """CSR arrays in (host), CSR arrays out (host): (indptr, indices, data)."""
        if n_cols is not None and n_cols != self.m:
            raise ValueError(f"matmul: dimension mismatch with signature (n,k={n_cols}),(k={self.m},m)->(n,m)")
        indptr = np.asarray(indptr)
        indices = np.asarray(indices)
        T = self.compute_dtype(np.asarray(data).dtype)
        data = np.ascontiguousarray(data, dtype=T)
        if indptr.dtype not in (np.int32, np.int64):
            indptr = indptr.astype(np.int64)
        indptr = np.ascontiguousarray(indptr)
        aj = np.ascontiguousarray(indices, dtype=np.int32) if indices.dtype != np.int32 else np.ascontiguousarray(indices)
        if indices.dtype != np.int32 and indices.size and (indices.min() < 0 or indices.max() >= self.m):
            raise ValueError("column index out of range")
        n = len(indptr) - 1
        if n >= STREAM_MIN_ROWS:  # large host matrices: chunked, overlapped upload/compute/download
            return self.project_stream(indptr, aj, data, order=order, out_index_dtype=out_index_dtype,
                                       _index_rule_arrays=(indptr, indices))
        if indptr.ndim != 1 or n < 0:
            raise ValueError("index pointer should be a 1-D array of at least one entry")
        if n >= 0 and (int(indptr[0]) < 0 or int(indptr[-1]) < int(indptr[0])):
            raise ValueError("index pointer values must start at a non-negative value and be non-decreasing")
        if aj.ndim != 1 or data.ndim != 1 or aj.size < int(indptr[-1]) or data.size < int(indptr[-1]):
            # scipy's check_format: "indices and data should have the same size" / "Last value of
            # index pointer should be less than the size of index and data arrays"
            raise ValueError("Last value of index pointer should be less than the size of index and data arrays")
        a = nat.CsrIn(n, nat.ptr(indptr).value, nat.idx_code(indptr.dtype), nat.ptr(aj).value,
                      nat.ptr(data).value, nat.val_code(T), int(indptr[-1] - indptr[0]) if n >= 0 else 0)
        code = nat.RP_ORDER_SORTED if order == "sorted" else nat.RP_ORDER_SCIPY
        out = {}

        def alloc(_user, n_rows, k, p_indptr, p_ityp, p_indices, p_jtyp, p_data):
            # rp_project's callback: the exact nnz is known, so scipy's index-dtype rule applies here
            try:
                dt = out_index_dtype
                if dt is None:
                    dt = scipy_result_index_dtype((indptr, indices), k)
                    if self.r_index_dtype == np.int64:
                        dt = np.dtype(np.int64)
                dt = np.dtype(dt)
                # recycled, already-faulted host memory: first-touch faults of fresh arrays would
                # cost more than the copies themselves (hostmem.py)
                out["Cp"] = hostmem.empty(n_rows + 1, dt)
                out["Cj"] = hostmem.empty(k, dt)
                out["Cx"] = hostmem.empty(k, T)
                p_indptr[0] = out["Cp"].ctypes.data
                p_indices[0] = out["Cj"].ctypes.data if k else None
                p_data[0] = out["Cx"].ctypes.data if k else None
                p_ityp[0] = p_jtyp[0] = nat.idx_code(dt)
                return 0
            except Exception:  # noqa: BLE001 - reported as RP_ERR_NOMEM by the library
                return 1

        cb = nat.ALLOC_FN(alloc)
        with self._lock:
            rc = self._lib.rp_project(self._h, ctypes.byref(a), code, cb, None)
        if rc == nat.RP_ERR_INVALID:
            raise ValueError(self._lib.rp_last_error().decode())
        nat.check(rc)
        return out["Cp"], out["Cj"], out["Cx"]

    def project_stream(self, indptr, indices, data, order: str = "scipy", chunk_rows: int = 0, out=None,
                       out_index_dtype=None, _index_rule_arrays=None):
        """Host CSR in -> host CSR out through ``rp_project_stream``: rows in chunks (default 2M)
        whose upload, projection and download overlap (boundary 2, BASELINE configs[1]'s chunked
        row streaming). ``out``: optional ``(indptr, indices, data)`` host arrays to fill (reused
        buffers avoid first-touch page faults; capacity = len(indices)); else recycled host memory
        sized from the expected nnz, with one exact retry if that was short. Returns
        ``(indptr, indices[:nnz], data[:nnz])``."""
        indptr = np.ascontiguousarray(indptr)
        if indptr.dtype not in (np.int32, np.int64):
            indptr = indptr.astype(np.int64)
        indices = np.asarray(indices)
        T = self.compute_dtype(np.asarray(data).dtype)
        data = np.ascontiguousarray(data, dtype=T)
        aj = np.ascontiguousarray(indices, dtype=np.int32)
        n = len(indptr) - 1
        if indptr.ndim != 1 or n < 0:
            raise ValueError("index pointer should be a 1-D array of at least one entry")
        nnz_a = int(indptr[-1]) - int(indptr[0])
        if int(indptr[0]) < 0 or nnz_a < 0 or aj.size < int(indptr[-1]) or data.size < int(indptr[-1]):
            raise ValueError("Last value of index pointer should be less than the size of index and data arrays")
        rule = _index_rule_arrays if _index_rule_arrays is not None else (indptr, indices)

        def alloc(cap, dt):
            dt = np.dtype(dt)
            return hostmem.empty(n + 1, dt), hostmem.empty(max(cap, 1), dt), hostmem.empty(max(cap, 1), T)

        keep_dt = None if out is None else np.dtype(out[0].dtype)  # a caller's out fixes the index dtype
        if out is None:
            exp = nnz_a * self.nnz / max(self.m, 1)
            cap = int(1.02 * exp + 8.0 * np.sqrt(exp + 1.0)) + 65536
            dt = out_index_dtype or (np.int64 if self.r_index_dtype == np.int64 else scipy_result_index_dtype(rule, cap))
            out = alloc(cap, dt)
        Cp, Cj, Cx = out
        a = nat.CsrIn(n, nat.ptr(indptr).value, nat.idx_code(indptr.dtype), nat.ptr(aj).value,
                      nat.ptr(data).value, nat.val_code(T), nnz_a)
        code = nat.RP_ORDER_SORTED if order == "sorted" else nat.RP_ORDER_SCIPY
        total = ctypes.c_int64(0)
        for attempt in range(2):
            if Cx.dtype != T or Cj.dtype != Cp.dtype or Cp.size != n + 1:
                raise ValueError("out arrays: indptr of n_rows + 1 entries, indices of indptr's dtype, data of "
                                 f"the compute dtype {T}")
            c = nat.CsrOut(nat.ptr(Cp).value, nat.idx_code(Cp.dtype), nat.ptr(Cj).value, nat.idx_code(Cj.dtype),
                           nat.ptr(Cx).value, int(Cj.size))
            with self._lock:
                rc = self._lib.rp_project_stream(self._h, ctypes.byref(a), code, int(chunk_rows), ctypes.byref(c),
                                                 ctypes.byref(total))
            k = int(total.value)
            if rc == nat.RP_ERR_CAPACITY and attempt == 0:
                dt = keep_dt or out_index_dtype or (np.int64 if self.r_index_dtype == np.int64
                                                    else scipy_result_index_dtype(rule, k))
                Cp, Cj, Cx = alloc(k, dt)
                continue
            if rc == nat.RP_ERR_INVALID:
                raise ValueError(self._lib.rp_last_error().decode())
            nat.check(rc)
            break
        if keep_dt is None and out_index_dtype is None and Cp.dtype == np.int64 and self.r_index_dtype != np.int64:
            want = scipy_result_index_dtype(rule, k)   # the estimate passed 2^31, the result did not
            if want != Cp.dtype:
                Cp, Cj = Cp.astype(want), Cj[:k].astype(want)
        return Cp, Cj[:k], Cx[:k]

    def stream_stats(self) -> dict:
        """What the last stream call (``project_stream`` / the libsvm stream) did
        (rp_project_stream_stats): chunks streamed, chunks recomputed after the pipeline because
        their output outgrew the device slot (0 in the steady state), slot capacities raised from
        the measured output per entry."""
        ch, rd, rg = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        nat.check(self._lib.rp_project_stream_stats(self._h, ctypes.byref(ch), ctypes.byref(rd), ctypes.byref(rg)))
        return {"chunks": int(ch.value), "recomputed": int(rd.value), "regrown": int(rg.value)}

    def matmul(self, A, order: str = "scipy"):
        """``A @ R`` for sparse A, returning what scipy returns (container of A's class)."""
        if not sp.issparse(A):
            raise TypeError("Projector.matmul expects a scipy sparse matrix/array")
        if A.shape[1] != self.m:
            raise ValueError(f"matmul: dimension mismatch with signature (n,k={A.shape[1]}),(k={self.m},m)->(n,m)")
        cls = A.__class__ if A.format == "csr" else (sp.csr_array if isinstance(A, sp.sparray) else sp.csr_matrix)
        Ac = A if A.format == "csr" else A.tocsr()
        T = self.compute_dtype(Ac.dtype)
        Cp, Cj, Cx = self.project_arrays(Ac.indptr, Ac.indices, Ac.data.astype(T, copy=False), order=order)
        return cls((Cx, Cj, Cp), shape=(Ac.shape[0], self.p))

    # -------------------------------------------------------------------------------- device path
    def project_device(self, Ap, Aj, Ax, Cp, Cj, Cx, order: str = "scipy", stream=0, workspace=None,
                       nnz_a: int = -1, sync: bool = True):
        """Device-resident product on raw device pointers or torch tensors. ``workspace``: a torch
        uint8 tensor (or a ``(pointer, bytes)`` pair) of ``workspace_bytes(n, nnz)``, or None.

        Returns the exact output nnz when ``sync`` (raises ``RPError`` with code RP_ERR_CAPACITY
        if ``Cj``/``Cx`` are too small; in auto staging mode the host reads the device's staging
        verdict and launches only the chosen branch), else None: the launch never waits on the host
        (the verdict gates the staged kernels on the device), so it can be captured in a graph when
        ``workspace`` is given and ``nnz_a >= 0``."""
        def p_(t):
            return int(t.data_ptr()) if hasattr(t, "data_ptr") else int(t)

        def code_(t, ints=True):
            dt = str(getattr(t, "dtype", ""))
            if ints:
                return nat.RP_I64 if dt.endswith("int64") else nat.RP_I32
            return nat.RP_F64 if dt.endswith("float64") else nat.RP_F32

        n = (Ap.numel() if hasattr(Ap, "numel") else len(Ap)) - 1
        cap = Cj.numel() if hasattr(Cj, "numel") else len(Cj)
        a = nat.CsrIn(n, p_(Ap), code_(Ap), p_(Aj), p_(Ax), code_(Ax, False), int(nnz_a))
        c = nat.CsrOut(p_(Cp), code_(Cp), p_(Cj), code_(Cj), p_(Cx), int(cap))
        total = ctypes.c_int64(0)
        code = nat.RP_ORDER_SORTED if order == "sorted" else nat.RP_ORDER_SCIPY
        if workspace is None:
            ws_ptr, ws_bytes = 0, 0
        elif hasattr(workspace, "data_ptr"):
            ws_ptr, ws_bytes = int(workspace.data_ptr()), int(workspace.numel() * workspace.element_size())
        else:
            ws_ptr, ws_bytes = int(workspace[0]), int(workspace[1])  # (device pointer, bytes)
        rc = self._lib.rp_project_device(self._h, ctypes.byref(a), ctypes.byref(c), code,
                                         ctypes.c_void_p(ws_ptr), ws_bytes,
                                         ctypes.c_void_p(stream), ctypes.byref(total) if sync else None)
        if rc == nat.RP_ERR_CAPACITY:
            # raised without a local name: a frame holding its own exception is a reference cycle
            # (frame -> exception -> traceback -> frame) that would keep the caller's output tensors
            # (tens of GB at full size) alive until a GC pass
            raise nat.capacity_error(rc, self._lib.rp_last_error().decode(), int(total.value))
        nat.check(rc)
        return int(total.value) if sync else None

    def workspace_bytes(self, n_rows: int, nnz_a: int = -1, dtype=None) -> int:
        """Device workspace for ``project_device`` on n_rows rows / nnz_a entries (staging included);
        ``dtype`` (the compute type, float32 or float64) sizes the value parts for it, else for
        float64."""
        if dtype is not None and nnz_a >= 0:
            # torch dtypes carry .itemsize; numpy dtypes / scalar types / strings go through np.dtype
            size = getattr(dtype, "itemsize", None)
            if not isinstance(size, int):
                size = np.dtype(dtype).itemsize
            code = nat.RP_F64 if size == 8 else nat.RP_F32
            return int(self._lib.rp_project_workspace_bytes_for(self._h, int(n_rows), int(nnz_a), code))
        return int(self._lib.rp_project_workspace_bytes(self._h, int(n_rows), int(nnz_a)))

    def plan(self, n_rows: int, nnz_a: int = -1) -> dict:
        """The kernel pipeline ``project_device`` runs for this shape with a full workspace
        (rp_project_plan): {"pipeline": "tile"|"rowlane", "staged": bool | "auto" (decided per call
        from a sample of the feature ids, see ``choice``), "bucket_shift": int}."""
        pipe, st, sb = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        nat.check(self._lib.rp_project_plan(self._h, int(n_rows), int(nnz_a), ctypes.byref(pipe), ctypes.byref(st),
                                            ctypes.byref(sb)))
        return {"pipeline": {0: "tile", 1: "rowlane"}[pipe.value],
                "staged": "auto" if st.value == 2 else bool(st.value), "bucket_shift": int(sb.value)}

    def choice(self, n_rows: int, nnz_a: int, workspace) -> bool:
        """After a completed ``project_device`` call with ``workspace`` (torch uint8 tensor): whether
        it ran the staged gather (auto mode decides per call from a sample taken on the device)."""
        st = ctypes.c_int32()
        ptr = int(workspace.data_ptr()) if hasattr(workspace, "data_ptr") else int(workspace)
        nat.check(self._lib.rp_project_choice(self._h, int(n_rows), int(nnz_a), ctypes.c_void_p(ptr), ctypes.byref(st)))
        return bool(st.value)

    def set_staging(self, mode: str = "auto", bucket_shift: int = 0):
        """Staged gather: "auto", "off" or "on" (identical results)."""
        code = {"auto": -1, "off": 0, "on": 1}[mode]
        nat.check(self._lib.rp_projector_set_staging(self._h, code, int(bucket_shift)))

    _OPTIONS = {"pipeline": nat.RP_OPT_PIPELINE, "defer_polls": nat.RP_OPT_DEFER_POLLS,
                "defer_ticks": nat.RP_OPT_DEFER_TICKS, "chunk_rows": nat.RP_OPT_CHUNK_ROWS,
                "host_threads": nat.RP_OPT_HOST_THREADS}
    _OPTION_DEFAULTS = {"pipeline": 0, "defer_polls": -2, "defer_ticks": -1, "chunk_rows": 0, "host_threads": -1}
    _PIPELINES = {"auto": 0, "tile": 1, "rowlane": 2}

    def set_option(self, name: str, value):
        """Tuning / test option of this projector (rp_projector_set_option; results are identical
        under every setting): pipeline ("auto" | "tile" | "rowlane"), defer_polls, defer_ticks,
        chunk_rows, host_threads; ``None`` restores the default."""
        if name not in self._OPTIONS:
            raise ValueError(f"unknown option {name!r}; one of {sorted(self._OPTIONS)}")
        if value is None:
            value = self._OPTION_DEFAULTS[name]
        elif name == "pipeline" and isinstance(value, str):
            value = self._PIPELINES[value]
        nat.check(self._lib.rp_projector_set_option(self._h, self._OPTIONS[name], int(value)))

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        nat.check(self._lib.rp_projector_get_option(self._h, self._OPTIONS[name], ctypes.byref(v)))
        return int(v.value)

    @contextlib.contextmanager
    def options(self, **kw):
        """Set options for the duration of a ``with`` block, then restore the previous values."""
        old = {k: self.get_option(k) for k in kw}
        try:
            for k, v in kw.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    def __repr__(self):
        return f"Projector(m={self.m}, p={self.p}, nnz={self.nnz}, layout={self.layout}, device={self.device})"


# ------------------------------------------------------------------------------------------------
# projector cache for the drop-ins: one upload per R object (the broadcast-once of the recipe)
_cache: "dict[int, tuple]" = {}
_cache_lock = threading.Lock()


def _fingerprint(R):
    if sp.issparse(R):
        arrs = [getattr(R, n, None) for n in ("data", "indices", "indptr")]
        ptrs = tuple((a.__array_interface__["data"][0], a.size) if isinstance(a, np.ndarray) else None for a in arrs)
        return (R.format, R.shape, R.nnz, str(R.dtype), ptrs)
    a = np.asarray(R)
    return ("dense", a.shape, str(a.dtype), a.__array_interface__["data"][0])


def get_projector(R, device: int = 0) -> Projector:
    """The resident projector for ``R`` (a scipy matrix, or a ``Projector`` passed through)."""
    if isinstance(R, Projector):
        return R
    key = id(R)
    fp = _fingerprint(R)
    with _cache_lock:
        hit = _cache.get(key)
        if hit is not None and hit[1] == fp and hit[2] == device:
            ref = hit[0]()
            if ref is not None:
                return hit[3]
    proj = Projector(R, device=device)
    try:
        ref = weakref.ref(R, lambda _r, k=key: _cache.pop(k, None))
    except TypeError:
        ref = lambda: R  # noqa: E731 - objects without weakref support stay cached
    with _cache_lock:
        _cache[key] = (ref, fp, device, proj)
    return proj
