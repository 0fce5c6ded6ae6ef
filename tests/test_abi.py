"""The C-ABI library (librp.so) loads without a GPU and exports every symbol include/rp.h declares."""
import ctypes
import os
import re

from conftest import ROOT
from randomprojection_amd import _native as nat


def _declared():
    src = open(os.path.join(ROOT, "include", "rp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rp_[a-z_]+)\s*\(", src)))


def test_header_matches_binding_table():
    assert _declared() == sorted(nat.EXPORTS)


def test_library_exports_all_symbols():
    lib = ctypes.CDLL(nat.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name


def test_calls_without_gpu_fail_loudly():
    lib = nat.load()
    assert lib.rp_version().startswith(b"rp-mi355x")
    n = ctypes.c_int(-1)
    rc = lib.rp_device_count(ctypes.byref(n))
    if rc != nat.RP_OK:                       # CPU container: error + message, never a crash
        assert n.value == 0 and lib.rp_last_error()


def test_invalid_arguments_rejected_before_device_use():
    lib = nat.load()
    h = ctypes.c_void_p()
    rc = lib.rp_projector_create(0, 10, 0, None, nat.RP_I32, None, nat.RP_I32, None, nat.RP_F32, 0, ctypes.byref(h))
    assert rc == nat.RP_ERR_INVALID and b"bad shape" in lib.rp_last_error()
    rc = lib.rp_projector_create(0, 10, 40000, None, nat.RP_I32, None, nat.RP_I32, None, nat.RP_F32, 0, ctypes.byref(h))
    assert rc in (nat.RP_ERR_INVALID, nat.RP_ERR_UNSUPPORTED)


def test_library_build_id_matches_sources():
    """The loaded librp carries the source id of the files it was compiled from (build.py), and it is
    the id of the sources on disk: the loader refuses anything else."""
    from randomprojection_amd import build

    nat.load()
    assert nat.build_id() == build.source_id() == build.library_id(nat.LIB_PATH)
    assert not build.needs_build()


def test_touched_source_is_a_stale_library(tmp_path):
    """A .hip file changed after the build makes the library stale: check_build_id raises."""
    import shutil

    from randomprojection_amd import build

    lib = nat.load()
    for rel in build.HASHED:
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(ROOT, rel), dst)
    assert nat.check_build_id(lib, str(tmp_path)) == build.source_id()
    with open(tmp_path / "randomprojection_amd" / "csrc" / "rp_spgemm.hip", "a") as f:
        f.write("// touched\n")
    try:
        nat.check_build_id(lib, str(tmp_path))
    except nat.StaleLibrary as e:
        assert "rebuild" in str(e)
    else:
        raise AssertionError("a touched source was not detected")


def test_source_id_covers_flags():
    """A compile flag (e.g. -ffp-contract, which the bit-exactness depends on) is part of the id."""
    from randomprojection_amd import build

    sid = build.source_id()
    build.FLAGS.append("-DRP_TEST_FLAG")
    try:
        assert build.source_id() != sid
    finally:
        build.FLAGS.pop()
    assert build.source_id() == sid


def test_committed_traffic_matches_sources():
    """profiles/traffic_latest.json (the PMC HBM bytes bench.py puts in roofline.traffic) was
    measured on the library built from the sources on disk: bench.py only uses it when its
    src_sha16 equals the loaded build id, so a source change without a re-profile shows up here
    rather than as a silent traffic=null in the round-end bench line."""
    import json

    from randomprojection_amd import build

    with open(os.path.join(ROOT, "profiles", "traffic_latest.json")) as f:
        tj = json.load(f)
    assert tj["src_sha16"] == build.source_id()
    assert tj["hbm_bytes_per_launch"] > 0


def test_source_id_follows_the_compiler_not_its_path(monkeypatch):
    """The id hashes what ``hipcc --version`` reports: the same compiler reached through another
    path keeps the id (no spurious rebuild), another compiler identity changes it."""
    from randomprojection_amd import build

    sid = build.source_id()
    real = os.path.realpath(build.HIPCC)
    assert build.compiler_identity(real) == build.compiler_identity()
    # the library records the identity it was built with: the loader recomputes the id from it
    # without running the compiler (a child process of a GPU-initialised process is refused on
    # the GPU box)
    assert build.library_cc(nat.LIB_PATH) == build.compiler_hash()
    assert build.source_id(cc=build.library_cc(nat.LIB_PATH)) == sid
    monkeypatch.setattr(build, "compiler_identity", lambda hipcc=None: "AMD clang version 0.0 (other)")
    assert build.source_id() != sid


def test_abi_version_matches_bindings():
    """rp_abi_version() equals include/rp.h's RP_ABI_VERSION and the bindings' ABI_VERSION (a changed
    signature under an old symbol name is refused at load time instead of passing garbage)."""
    src = open(os.path.join(ROOT, "include", "rp.h")).read()
    want = int(re.search(r"#define RP_ABI_VERSION (\d+)", src).group(1))
    assert nat.load().rp_abi_version() == want == nat.ABI_VERSION
