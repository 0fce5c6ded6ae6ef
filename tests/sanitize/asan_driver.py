"""Runs inside a child process with clang's ASan runtime preloaded (tests/test_sanitizers.py): the
host code of librp (ASan + UBSan build, tests/sanitize/_build/librp_asan.so) and the C oracle
(_build/liboracle_smmp_asan.so) on the cases the parent wrote to an .npz, results to another .npz.
Every array handed to the native code has exactly the size the C-ABI documents, so any read or
write past it is an ASan report (the child aborts with a non-zero status).

    python asan_driver.py <librp_asan.so> <cases.npz> <out.npz> [gpu]
    python asan_driver.py <librp_asan.so> canary     (must be caught: an R whose indptr promises
                                                      one more entry than its index array holds)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

RP_I32, RP_I64, RP_F32, RP_F64 = 1, 2, 3, 4


class Info(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("p", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("layout", ctypes.c_int32), ("value_type", ctypes.c_int32), ("magnitude", ctypes.c_double),
                ("block_shift", ctypes.c_int32), ("n_buffers", ctypes.c_int32),
                ("buffer_bytes", ctypes.c_int64 * 4)]


def code(a):
    return {np.dtype(np.int32): RP_I32, np.dtype(np.int64): RP_I64, np.dtype(np.float32): RP_F32,
            np.dtype(np.float64): RP_F64}[a.dtype]


def vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


def canary(lib):
    ip = np.array([0, 2, 5], np.int32)
    ix = np.array([1, 3, 0, 2], np.int32)  # 4 entries, indptr says 5
    dx = np.ones(5, np.float32)
    info = Info()
    lib.rp_pack_r_host(ctypes.c_int64(2), ctypes.c_int64(4), vp(ip), RP_I32, vp(ix), RP_I32, vp(dx), RP_F32, 0,
                       ctypes.byref(info), None, None, None)


def main():
    lib = ctypes.CDLL(sys.argv[1])
    lib.rp_last_error.restype = ctypes.c_char_p
    vpt, i32, i64, P = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER
    lib.rp_projector_create.argtypes = [ctypes.c_int, i64, i64, vpt, i32, vpt, i32, vpt, i32, i32, P(vpt)]
    lib.rp_project_host_begin.argtypes = [vpt, P(CsrIn), i32, P(vpt), P(i64)]
    lib.rp_result_fetch.argtypes = [vpt, vpt, i32, vpt, i32, vpt]
    lib.rp_result_free.argtypes = [vpt]
    lib.rp_project_stream.argtypes = [vpt, P(CsrIn), i32, i64, P(CsrOut), P(i64)]
    lib.rp_libsvm_project_stream.argtypes = [vpt, vpt, i64, i32, i64, vpt, i64, P(CsrOut), P(i64), P(i64), P(i64)]
    lib.rp_projector_destroy.argtypes = [vpt]
    if sys.argv[2] == "canary":
        canary(lib)
        return
    cases = np.load(sys.argv[2], allow_pickle=False)
    out = {}
    # ---- librp host code: rp_pack_r_host (R validation, layout choice, packing) on every R case,
    # sizes first (NULL buffers), then exact-size buffers
    for name in sorted({k.split("/")[1] for k in cases.files if k.startswith("pack/")}):
        g = lambda f: cases[f"pack/{name}/{f}"]  # noqa: E731
        ip, ix, dx = g("indptr"), g("indices"), g("data")
        m, p, layout = int(g("m")), int(g("p")), int(g("layout"))
        info = Info()
        rc = lib.rp_pack_r_host(ctypes.c_int64(m), ctypes.c_int64(p), vp(ip), code(ip), vp(ix), code(ix), vp(dx),
                                code(dx), layout, ctypes.byref(info), None, None, None)
        out[f"pack/{name}/rc"] = np.array([rc])
        if rc == 0:
            bufs = [np.zeros(max(int(info.buffer_bytes[i]), 0), np.uint8) for i in range(3)]
            info2 = Info()
            rc2 = lib.rp_pack_r_host(ctypes.c_int64(m), ctypes.c_int64(p), vp(ip), code(ip), vp(ix), code(ix),
                                     vp(dx), code(dx), layout, ctypes.byref(info2), *[vp(b) for b in bufs])
            out[f"pack/{name}/rc2"] = np.array([rc2])
            out[f"pack/{name}/layout"] = np.array([info2.layout])
            for i, b in enumerate(bufs):
                out[f"pack/{name}/buf{i}"] = b
        else:
            out[f"pack/{name}/err"] = np.frombuffer(lib.rp_last_error() or b"-", np.uint8)
    # ---- argument validation of the entry points that take host arrays (no device needed)
    out["null/stream"] = np.array([lib.rp_project_stream(None, None, 0, ctypes.c_int64(0), None, None)])
    out["null/libsvm"] = np.array([lib.rp_libsvm_project_stream(None, None, ctypes.c_int64(0), 0, ctypes.c_int64(0),
                                                                 None, ctypes.c_int64(0), None, None, None, None)])
    out["null/begin"] = np.array([lib.rp_project_host_begin(None, None, 0, None, None)])
    # ---- the C oracle (ASan + UBSan build) on the golden cases
    from oracle import smmp  # ORACLE_SMMP_LIB points it at the sanitizer build
    from conftest import golden_R, golden_csr
    gold = np.load(os.path.join(ROOT, "tests", "golden", "golden_v1.npz"), allow_pickle=False)
    for name in gold["cases"]:
        A = golden_csr(gold, "A_" + str(name))
        R = golden_R(gold, int(gold["R_" + str(name)][0]))
        Cp, Cj, Cx, _, _ = smmp.matmat(A, R)
        out[f"oracle/{name}/indptr"], out[f"oracle/{name}/indices"], out[f"oracle/{name}/data"] = Cp, Cj, Cx
    if len(sys.argv) > 4 and sys.argv[4] == "gpu":
        gpu_paths(lib, cases, out)
    np.savez(sys.argv[3], **out)


class CsrIn(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("indptr", ctypes.c_void_p), ("indptr_type", ctypes.c_int32),
                ("indices", ctypes.c_void_p), ("data", ctypes.c_void_p), ("data_type", ctypes.c_int32),
                ("nnz", ctypes.c_int64)]


class CsrOut(ctypes.Structure):
    _fields_ = [("indptr", ctypes.c_void_p), ("indptr_type", ctypes.c_int32), ("indices", ctypes.c_void_p),
                ("indices_type", ctypes.c_int32), ("data", ctypes.c_void_p), ("capacity", ctypes.c_int64)]


def gpu_paths(lib, cases, out):
    """On a GPU box: the host sides of the projector upload, the host-buffer path (begin / fetch), the
    chunked stream and the libsvm stream, every host array of exactly its documented size."""
    from conftest import golden_R, golden_csr

    gold = np.load(os.path.join(ROOT, "tests", "golden", "golden_v1.npz"), allow_pickle=False)
    R = golden_R(gold, 1).tocsr()
    A = golden_csr(gold, "A_kdd_vals").astype(np.float32)
    i64, P = ctypes.c_int64, ctypes.POINTER
    h = ctypes.c_void_p()
    rc = lib.rp_projector_create(0, i64(R.shape[0]), i64(R.shape[1]), vp(R.indptr), code(R.indptr), vp(R.indices),
                                 code(R.indices), vp(R.data), code(R.data), 0, ctypes.byref(h))
    assert rc == 0, lib.rp_last_error()
    n = A.shape[0]
    for ipt in (np.int32, np.int64):
        ap, aj, ax = A.indptr.astype(ipt), A.indices.astype(np.int32), A.data
        a = CsrIn(n, vp(ap), code(ap), vp(aj), vp(ax), RP_F32, int(A.nnz))
        # host begin / fetch
        res, nnz = ctypes.c_void_p(), i64(0)
        assert lib.rp_project_host_begin(h, ctypes.byref(a), 0, ctypes.byref(res), ctypes.byref(nnz)) == 0
        cp, cj, cx = np.empty(n + 1, np.int64), np.empty(nnz.value, np.int32), np.empty(nnz.value, np.float32)
        assert lib.rp_result_fetch(res, vp(cp), RP_I64, vp(cj), RP_I32, vp(cx)) == 0
        lib.rp_result_free(res)
        tag = np.dtype(ipt).name
        out[f"gpu/begin_{tag}/indptr"], out[f"gpu/begin_{tag}/indices"], out[f"gpu/begin_{tag}/data"] = cp, cj, cx
        # chunked stream, many small chunks, exact-size outputs
        sp_, sj, sx = np.empty(n + 1, ipt), np.empty(nnz.value, np.int32), np.empty(nnz.value, np.float32)
        c = CsrOut(vp(sp_), code(sp_), vp(sj), RP_I32, vp(sx), nnz.value)
        tot = i64(0)
        assert lib.rp_project_stream(h, ctypes.byref(a), 0, i64(97), ctypes.byref(c), ctypes.byref(tot)) == 0
        out[f"gpu/stream_{tag}/indptr"], out[f"gpu/stream_{tag}/indices"], out[f"gpu/stream_{tag}/data"] = sp_, sj, sx
    # libsvm text of the same rows (1-based features), exactly its bytes, chunked small; once with and
    # once without the final newline
    lines = []
    for r in range(n):
        b, e = A.indptr[r], A.indptr[r + 1]
        lines.append(" ".join([str(r % 2)] + [f"{j + 1}:{float(v)!r}" for j, v in zip(A.indices[b:e], A.data[b:e])]))
    for tail in ("\n", ""):
        text = np.frombuffer(("\n".join(lines) + tail).encode(), np.uint8).copy()
        buf = np.zeros(text.size + 16, np.uint8)  # 16-byte aligned start (rp_libsvm_parse_device)
        off = (-buf.ctypes.data) % 16
        t = buf[off:off + text.size]
        t[:] = text
        nnz_c = int(out["gpu/begin_int32/indices"].size)
        labels = np.empty(n, np.float64)
        lp, lj, lx = np.empty(n + 1, np.int64), np.empty(nnz_c, np.int32), np.empty(nnz_c, np.float32)
        c = CsrOut(vp(lp), RP_I64, vp(lj), RP_I32, vp(lx), nnz_c)
        nr, tot, el = i64(0), i64(0), i64(-1)
        rc = lib.rp_libsvm_project_stream(h, vp(t), i64(t.size), 0, i64(4096), vp(labels), i64(n), ctypes.byref(c),
                                          ctypes.byref(nr), ctypes.byref(tot), ctypes.byref(el))
        assert rc == 0 and nr.value == n and tot.value == nnz_c, (rc, lib.rp_last_error())
        k = "nl" if tail else "nonl"
        out[f"gpu/libsvm_{k}/indptr"], out[f"gpu/libsvm_{k}/indices"], out[f"gpu/libsvm_{k}/data"] = lp, lj, lx
        out[f"gpu/libsvm_{k}/labels"] = labels
    lib.rp_projector_destroy(h)


if __name__ == "__main__":
    main()
