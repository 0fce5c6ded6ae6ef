"""ctypes binding of librp.so (include/rp.h). The product has no CPU fallback: if the library or a
GPU is missing, every compute call raises ``NativeUnavailable``/``RPError`` loudly."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librp.so")

RP_OK, RP_ERR_INVALID, RP_ERR_HIP, RP_ERR_CAPACITY, RP_ERR_UNSUPPORTED, RP_ERR_NOMEM, RP_ERR_TIMEOUT = range(7)
RP_I32, RP_I64, RP_F32, RP_F64, RP_BF16 = 1, 2, 3, 4, 5
RP_LAYOUT_AUTO, RP_LAYOUT_GENERIC, RP_LAYOUT_PACKED = 0, 1, 2
RP_ORDER_SCIPY, RP_ORDER_SORTED = 0, 1
RP_OPT_PIPELINE, RP_OPT_DEFER_POLLS, RP_OPT_DEFER_TICKS, RP_OPT_CHUNK_ROWS, RP_OPT_HOST_THREADS = 1, 2, 3, 4, 5
# include/rp.h RP_ABI_VERSION these bindings are written against (signatures below)
ABI_VERSION = 6

# every symbol include/rp.h declares (tests/test_abi.py checks the .so exports them all)
EXPORTS = (
    "rp_last_error", "rp_version", "rp_abi_version", "rp_build_id", "rp_device_count",
    "rp_projector_create", "rp_projector_info_get", "rp_projector_export",
    "rp_projector_create_from_device", "rp_projector_destroy", "rp_pack_r_host",
    "rp_project_workspace_bytes", "rp_project_workspace_bytes_for", "rp_project_plan", "rp_project_choice", "rp_projector_set_staging",
    "rp_projector_set_option", "rp_projector_get_option", "rp_project_device",
    "rp_project_host_begin", "rp_result_fetch", "rp_result_free", "rp_project",
    "rp_synth_rows_device", "rp_libsvm_parse_device", "rp_libsvm_project_stream", "rp_synth_libsvm_device", "rp_project_stream", "rp_project_stream_stats", "rp_host_alloc", "rp_host_free",
    "rp_dense_project_device",
)


class NativeUnavailable(RuntimeError):
    pass


class StaleLibrary(NativeUnavailable):
    """librp.so was built from other sources than the ones on disk (build.py source_id)."""


class RPError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"librp error {code}: {msg}")
        self.code = code


class ProjectorInfo(ctypes.Structure):
    _fields_ = [
        ("m", ctypes.c_int64), ("p", ctypes.c_int64), ("nnz", ctypes.c_int64),
        ("layout", ctypes.c_int32), ("value_type", ctypes.c_int32),
        ("magnitude", ctypes.c_double), ("block_shift", ctypes.c_int32),
        ("n_buffers", ctypes.c_int32), ("buffer_bytes", ctypes.c_int64 * 4),
    ]


class CsrIn(ctypes.Structure):
    _fields_ = [
        ("n_rows", ctypes.c_int64), ("indptr", ctypes.c_void_p), ("indptr_type", ctypes.c_int32),
        ("indices", ctypes.c_void_p), ("data", ctypes.c_void_p), ("data_type", ctypes.c_int32),
        ("nnz", ctypes.c_int64),
    ]


class CsrOut(ctypes.Structure):
    _fields_ = [
        ("indptr", ctypes.c_void_p), ("indptr_type", ctypes.c_int32),
        ("indices", ctypes.c_void_p), ("indices_type", ctypes.c_int32),
        ("data", ctypes.c_void_p), ("capacity", ctypes.c_int64),
    ]


# int (*rp_alloc_fn)(void* user, int64_t n_rows, int64_t nnz, void** indptr, int32_t* indptr_type,
#                    void** indices, int32_t* indices_type, void** data)
ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(ctypes.c_void_p))

_lib = None


_lib_path = None


def check_build_id(lib, root: str = None) -> str:
    """The library's source id (rp_build_id) if it equals the id of the sources under ``root``
    (default: this checkout); else ``StaleLibrary``."""
    from . import build as _build

    have = lib.rp_build_id().decode()
    # the compiler identity recorded in the binary at build time (no compiler run here)
    cc = _build.library_cc(getattr(lib, "_name", None) or LIB_PATH)
    if cc is None:
        raise StaleLibrary("librp carries no compiler identity: rebuild it (python -m randomprojection_amd.build)")
    want = _build.source_id(root or _build.ROOT, cc=cc)
    if have != want:
        raise StaleLibrary(f"librp was built from sources {have}, the sources on disk are {want}: rebuild it "
                           "(python -m randomprojection_amd.build); numbers from a stale binary are refused")
    return have


def build_id() -> str:
    """Source id of the loaded library (checked against the sources when it was loaded)."""
    return load().rp_build_id().decode()


def loaded_path() -> str:
    load()
    return _lib_path


def load(path: str = None, verify: bool = None):
    """Load librp.so (built by ``randomprojection_amd.build`` / ``__graft_entry__.build``) and check
    that it was built from the sources on disk. ``path``: another build (A/B timing scripts only;
    its id is reported, not checked unless ``verify``)."""
    global _lib, _lib_path
    if _lib is not None:
        if path is not None and os.path.abspath(path) != _lib_path:
            raise NativeUnavailable(f"librp already loaded from {_lib_path}, cannot load {path} too")
        return _lib
    if verify is None:
        verify = path is None
    if path is None:
        path = LIB_PATH
    if not os.path.exists(path):
        raise NativeUnavailable(
            f"{path} is missing: build it with `python -m randomprojection_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # torch wheels bundle their own libamdhip64.so.7 (+ HSA runtime). If librp pulled in
    # /opt/rocm's copy first, torch's later CUDA init would fail ("No HIP GPUs are available").
    # Importing torch first makes librp bind to the runtime already in the process (same SONAME),
    # so exactly one HIP runtime exists whichever side touches the GPU first.
    try:
        import torch  # noqa: F401
    except Exception:  # noqa: BLE001 - torch is optional for the host drop-ins
        pass
    lib = ctypes.CDLL(path)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    P = ctypes.POINTER
    sig = {
        "rp_last_error": (ctypes.c_char_p, []),
        "rp_version": (ctypes.c_char_p, []),
        "rp_abi_version": (ctypes.c_int, []),
        "rp_build_id": (ctypes.c_char_p, []),
        "rp_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "rp_projector_create": (ctypes.c_int, [ctypes.c_int, i64, i64, vp, i32, vp, i32, vp, i32, i32, P(vp)]),
        "rp_projector_info_get": (ctypes.c_int, [vp, P(ProjectorInfo)]),
        "rp_projector_export": (ctypes.c_int, [vp, i32, vp, vp]),
        "rp_projector_create_from_device": (ctypes.c_int, [ctypes.c_int, P(ProjectorInfo), P(vp), P(vp)]),
        "rp_projector_destroy": (ctypes.c_int, [vp]),
        "rp_pack_r_host": (ctypes.c_int, [i64, i64, vp, i32, vp, i32, vp, i32, i32, P(ProjectorInfo), vp, vp, vp]),
        "rp_project_workspace_bytes": (i64, [vp, i64, i64]),
        "rp_project_workspace_bytes_for": (i64, [vp, i64, i64, i32]),
        "rp_project_plan": (ctypes.c_int, [vp, i64, i64, P(i32), P(i32), P(i32)]),
        "rp_project_choice": (ctypes.c_int, [vp, i64, i64, vp, P(i32)]),
        "rp_projector_set_staging": (ctypes.c_int, [vp, i32, i32]),
        "rp_projector_set_option": (ctypes.c_int, [vp, i32, i64]),
        "rp_projector_get_option": (ctypes.c_int, [vp, i32, P(i64)]),
        "rp_project_device": (ctypes.c_int, [vp, P(CsrIn), P(CsrOut), i32, vp, i64, vp, P(i64)]),
        "rp_project_host_begin": (ctypes.c_int, [vp, P(CsrIn), i32, P(vp), P(i64)]),
        "rp_result_fetch": (ctypes.c_int, [vp, vp, i32, vp, i32, vp]),
        "rp_result_free": (ctypes.c_int, [vp]),
        "rp_project": (ctypes.c_int, [vp, P(CsrIn), i32, ALLOC_FN, vp]),
        "rp_project_stream": (ctypes.c_int, [vp, P(CsrIn), i32, i64, P(CsrOut), P(i64)]),
        "rp_project_stream_stats": (ctypes.c_int, [vp, P(i64), P(i64), P(i64)]),
        "rp_host_alloc": (ctypes.c_int, [i64, P(vp)]),
        "rp_host_free": (ctypes.c_int, [vp]),
        "rp_synth_rows_device": (ctypes.c_int, [ctypes.c_int, i64, i64, dbl, i32, i32, dbl, ctypes.c_uint64,
                                                vp, i32, vp, vp, vp, P(i64)]),
        "rp_dense_project_device": (ctypes.c_int, [ctypes.c_int, vp, i32, i64, i64, vp, i64, vp, i64, vp, i32]),
        "rp_libsvm_parse_device": (ctypes.c_int, [ctypes.c_int, vp, i64, i64, vp, vp, i32, vp, vp, i64, i64, vp,
                                                  P(i64), P(i64), P(i64)]),
        "rp_libsvm_project_stream": (ctypes.c_int, [vp, vp, i64, i32, i64, vp, i64, P(CsrOut), P(i64), P(i64),
                                                    P(i64)]),
        "rp_synth_libsvm_device": (ctypes.c_int, [ctypes.c_int, i64, vp, vp, ctypes.c_uint64, vp, vp, i64, vp,
                                                  P(i64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name, None)
        if f is None:
            raise NativeUnavailable(f"{path} does not export {name}: rebuild it")
        f.restype = res
        f.argtypes = args
    if lib.rp_abi_version() != ABI_VERSION:
        raise NativeUnavailable(f"{path} has ABI version {lib.rp_abi_version()}, these bindings are written "
                                f"against {ABI_VERSION} (include/rp.h RP_ABI_VERSION): rebuild or update them")
    if verify:
        check_build_id(lib)
    _lib, _lib_path = lib, os.path.abspath(path)
    return lib


def capacity_error(code: int, msg: str, nnz: int) -> RPError:
    """RP_ERR_CAPACITY as an exception carrying the exact nnz the output needs."""
    e = RPError(code, msg)
    e.nnz = nnz
    return e


def check(rc: int):
    if rc != RP_OK:
        raise RPError(rc, load().rp_last_error().decode(errors="replace"))


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = load().rp_device_count(ctypes.byref(n))
    return n.value if rc == RP_OK else 0


def idx_code(dtype) -> int:
    dtype = np.dtype(dtype)
    if dtype == np.int32:
        return RP_I32
    if dtype == np.int64:
        return RP_I64
    raise TypeError(f"index dtype must be int32 or int64, got {dtype}")


def val_code(dtype) -> int:
    dtype = np.dtype(dtype)
    if dtype == np.float32:
        return RP_F32
    if dtype == np.float64:
        return RP_F64
    raise TypeError(f"value dtype must be float32 or float64, got {dtype}")


def ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(a.ctypes.data or 0)
