"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race detection /
sanitizers": host ASan/UBSan on the C++ CPU restatement). tests/sanitize/Makefile builds librp
(device code as usual, host code instrumented: -Xarch_host -fsanitize=...) and the C oracle with
clang's sanitizers; tests/sanitize/asan_driver.py runs them in a child process with the ASan
runtime preloaded, on exact-size arrays, so a host read or write past a documented size aborts
the child. Results must equal those of the normal builds."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import ROOT, golden_R, same_bits

SAN = os.path.join(ROOT, "tests", "sanitize")
BUILD = os.path.join(SAN, "_build")


def _runtime(name):
    hits = sorted(glob.glob(f"/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.{name}-x86_64.so"))
    return hits[-1] if hits else None


@pytest.fixture(scope="module")
def asan_libs():
    rt = _runtime("asan")
    if rt is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no ROCm clang ASan runtime / hipcc in this image")
    subprocess.run(["make", "-s", "-j3", "-C", SAN], check=True, stdout=subprocess.DEVNULL)
    return rt, os.path.join(BUILD, "librp_asan.so"), os.path.join(BUILD, "liboracle_smmp_asan.so")


def _r_cases(golden):
    """R operands for rp_pack_r_host: the golden ones (f32 / f64, CSC -> CSR), edge shapes (empty rows,
    rows of > 4 entries: long-row records, p = 16384 (packed) and 32767 (generic), int64 indptr and
    indices, one zero value), and invalid ones (column out of range, decreasing indptr)."""
    rng = np.random.default_rng(5)
    cases = {}

    def add(name, R, layout=0, ip=np.int32, ix=np.int32):
        R = sp.csr_matrix(R)
        cases[name] = dict(indptr=R.indptr.astype(ip), indices=R.indices.astype(ix), data=R.data,
                           m=np.array(R.shape[0]), p=np.array(R.shape[1]), layout=np.array(layout))

    for w in (1, 2):
        add(f"golden{w}", golden_R(golden, w).tocsr())
    mag = np.float32(1.3436618)
    for p, ip in ((16384, np.int64), (32767, np.int32)):
        m = 3000
        cnt = rng.choice([0, 0, 1, 2, 3, 6, 9], size=m)
        rows = np.repeat(np.arange(m), cnt)
        cols = np.concatenate([np.sort(rng.choice(p, size=k, replace=False)) for k in cnt])
        vals = np.where(rng.random(rows.size) < 0.5, -mag, mag).astype(np.float32)
        add(f"p{p}", sp.csr_matrix((vals, (rows, cols)), shape=(m, p)), ip=ip, ix=np.int64)
    R = sp.random(500, 64, density=0.05, random_state=1, format="csr", dtype=np.float32)
    R.data[:] = mag
    R.data[3] = 0.0
    add("zero_value", R)
    bad = dict(cases["golden1"])
    bad["indices"] = bad["indices"].copy()
    bad["indices"][7] = int(bad["p"]) + 3
    cases["bad_column"] = bad
    dec = dict(cases["golden1"])
    dec["indptr"] = dec["indptr"].copy()
    dec["indptr"][5] = dec["indptr"][6] + 1
    cases["bad_indptr"] = dec
    return cases


def _env(rt, liboracle_asan=None):
    # the sanitizer runtime first; whatever the environment already preloads stays after it
    pre = ":".join(x for x in (rt, os.environ.get("LD_PRELOAD", "")) if x)
    env = dict(os.environ, LD_PRELOAD=pre, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    if liboracle_asan:
        env["ORACLE_SMMP_LIB"] = liboracle_asan
    return env


def test_sanitizer_catches_a_host_overflow(asan_libs):
    """The harness works: an R whose indptr promises one more entry than its index array holds
    makes rp_pack_r_host read past the array, and the instrumented build reports it."""
    rt, librp_asan, liboracle_asan = asan_libs
    r = subprocess.run([sys.executable, os.path.join(SAN, "asan_driver.py"), librp_asan, "canary"],
                       env=_env(rt, liboracle_asan), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "AddressSanitizer: heap-buffer-overflow" in r.stderr, r.stderr[-2000:]


def test_host_code_under_asan_ubsan(asan_libs, golden, tmp_path):
    import ctypes

    from randomprojection_amd import _native as nat

    rt, librp_asan, liboracle_asan = asan_libs
    rcases = _r_cases(golden)
    flat = {f"pack/{n}/{k}": v for n, c in rcases.items() for k, v in c.items()}
    np.savez(tmp_path / "cases.npz", **flat)
    env = _env(rt, liboracle_asan)
    r = subprocess.run([sys.executable, os.path.join(SAN, "asan_driver.py"), librp_asan, str(tmp_path / "cases.npz"),
                        str(tmp_path / "out.npz")], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    got = np.load(tmp_path / "out.npz", allow_pickle=False)
    # the same calls on the normal build give the same codes and bytes
    lib = nat.load()
    for name, c in rcases.items():
        info = nat.ProjectorInfo()
        args = [ctypes.c_int64(int(c["m"])), ctypes.c_int64(int(c["p"])), c["indptr"].ctypes.data,
                nat.idx_code(c["indptr"].dtype), c["indices"].ctypes.data, nat.idx_code(c["indices"].dtype),
                c["data"].ctypes.data, nat.RP_F64 if c["data"].dtype == np.float64 else nat.RP_F32, int(c["layout"])]
        rc = lib.rp_pack_r_host(*args, ctypes.byref(info), None, None, None)
        assert int(got[f"pack/{name}/rc"][0]) == rc, name
        if name.startswith("bad"):
            assert rc == nat.RP_ERR_INVALID, name
        if rc:
            continue
        bufs = [np.zeros(int(info.buffer_bytes[i]), np.uint8) for i in range(3)]
        assert lib.rp_pack_r_host(*args, ctypes.byref(info), *[b.ctypes.data if b.size else None for b in bufs]) == 0
        assert int(got[f"pack/{name}/layout"][0]) == info.layout, name
        for i in range(3):
            assert np.array_equal(got[f"pack/{name}/buf{i}"], bufs[i]), (name, i)
    assert int(got["pack/p16384/layout"][0]) == nat.RP_LAYOUT_PACKED
    assert int(got["pack/p32767/layout"][0]) == nat.RP_LAYOUT_GENERIC
    assert int(got["pack/zero_value/layout"][0]) == nat.RP_LAYOUT_GENERIC
    for k in ("null/stream", "null/libsvm", "null/begin"):
        assert int(got[k][0]) == nat.RP_ERR_INVALID, k
    # the sanitizer build of the oracle reproduces the golden scipy products bit for bit
    for name in golden["cases"]:
        assert np.array_equal(got[f"oracle/{name}/indptr"], golden[f"C_{name}_indptr"])
        assert np.array_equal(got[f"oracle/{name}/indices"], golden[f"C_{name}_indices"])
        assert same_bits(got[f"oracle/{name}/data"], golden[f"C_{name}_data"])


@pytest.fixture(scope="module")
def ubsan_lib():
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc in this image")
    lib = os.path.join(BUILD, "librp_ubsan.so")
    srcs = glob.glob(os.path.join(ROOT, "randomprojection_amd", "csrc", "*")) + [os.path.join(ROOT, "include", "rp.h")]
    # the GPU box gets the built library but not its objects (.gpurunignore): use it when it is newer
    # than every source, else build (make would rebuild from the missing objects)
    if not (os.path.exists(lib) and os.path.getmtime(lib) > max(os.path.getmtime(f) for f in srcs)):
        subprocess.run(["make", "-s", "-j3", "-C", SAN, "_build/librp_ubsan.so"], check=True, stdout=subprocess.DEVNULL)
    return lib


@pytest.mark.gpu
def test_host_paths_under_ubsan_on_gpu(ubsan_lib, golden, tmp_path):
    """On the GPU box, the host code under UBSan (the ASan allocator could not map its heap beside the
    HIP runtime there: 'AddressSanitizer: out of memory' on a 4 MB runtime allocation, so ASan
    covers the host paths the CPU can reach, above) through the projector upload, the host-buffer
    path (begin / fetch), the chunked stream (int32 and int64 indptr, 97-row chunks) and the libsvm
    stream (4 KB chunks, text with and without its final newline), every host array of exactly its
    documented size: no UBSan report, and the results equal the oracle's product."""
    from oracle import smmp

    from conftest import golden_csr

    rt = _runtime("ubsan_standalone")
    if rt is None:
        pytest.skip("no UBSan runtime in this image")
    np.savez(tmp_path / "cases.npz", none=np.zeros(1))
    r = subprocess.run([sys.executable, "-u", os.path.join(SAN, "asan_driver.py"), ubsan_lib,
                        str(tmp_path / "cases.npz"), str(tmp_path / "out.npz"), "gpu"],
                       env=_env(rt), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    got = np.load(tmp_path / "out.npz", allow_pickle=False)
    A = golden_csr(golden, "A_kdd_vals").astype(np.float32)
    Cp, Cj, Cx, _, _ = smmp.matmat(A, golden_R(golden, 1).tocsr())
    for k in ("begin_int32", "begin_int64", "stream_int32", "stream_int64", "libsvm_nl", "libsvm_nonl"):
        assert np.array_equal(got[f"gpu/{k}/indptr"].astype(np.int64), Cp.astype(np.int64)), k
        assert np.array_equal(got[f"gpu/{k}/indices"], Cj.astype(np.int32)), k
        assert same_bits(got[f"gpu/{k}/data"], Cx), k
    assert np.array_equal(got["gpu/libsvm_nl/labels"], np.arange(A.shape[0]) % 2)
