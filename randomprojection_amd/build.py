"""Build librp.so (HIP, gfx950) in-tree with hipcc. No CUDA, no hipify, no multi-target build.

Every build embeds the sha256 prefix of its sources (``source_id``) as ``RP_SRC_SHA16``; the
library returns it from ``rp_build_id()`` and carries it behind a marker in the binary. A build is
needed exactly when that id differs from the sources on disk (not by file times), and the loader
(``_native.load``) refuses a library whose id does not match, so no number is ever measured on a
stale binary under a fresh source hash."""
from __future__ import annotations

import fcntl
import functools
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", n) for n in ("rp_spgemm.hip", "rp_libsvm.hip", "rp_dense.hip")]
# every file the compile reads (relative to the repo root): the id covers all of them
DEPS = ["randomprojection_amd/csrc/rp_spgemm.hip", "randomprojection_amd/csrc/rp_libsvm.hip",
        "randomprojection_amd/csrc/rp_dense.hip", "randomprojection_amd/csrc/rp_common.h",
        "randomprojection_amd/csrc/rp_pow5.h", "include/rp.h"]
OUT = os.path.join(HERE, "librp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    # scipy's csr_matmat rounds the multiply and the add separately: never contract to FMA
    "-ffp-contract=off", "-fno-fast-math", "-Wall",
]
MARKER = b"rp-src-sha16:"
CC_MARKER = b"rp-cc-sha16:"
HASHED = DEPS + ["randomprojection_amd/build.py"]  # files source_id covers (plus the compiler and FLAGS)


@functools.lru_cache(maxsize=None)
def compiler_identity(hipcc: str = None) -> str:
    """What ``hipcc --version`` reports (HIP and clang versions, target, install dir): the compiler
    itself, not the path or environment variable that named it. Only builds run it (a loader must
    not start a child process: under a GPU profiler the process has initialised the GPU already)."""
    try:
        out = subprocess.run([hipcc or HIPCC, "--version"], capture_output=True, text=True, timeout=60)
        return out.stdout.strip() if out.returncode == 0 else f"hipcc failed ({out.returncode})"
    except (OSError, subprocess.TimeoutExpired) as e:
        return f"hipcc unavailable ({type(e).__name__})"


def compiler_hash(hipcc: str = None) -> str:
    """16-hex-digit sha256 prefix of ``compiler_identity``; builds embed it in the library
    (``RP_CC_SHA16``) so that a loader can recompute the source id without running the compiler."""
    return hashlib.sha256(compiler_identity(hipcc).encode()).hexdigest()[:16]


def source_id(root: str = ROOT, cc: str = None) -> str:
    """sha256 prefix over (path, contents) of every source file of librp under ``root``, plus the
    compiler's identity hash ``cc`` (default: the compiler HIPCC names now, ``compiler_hash``), the
    flags and this build script: a changed flag such as -ffp-contract, which the bit-exactness
    depends on, or another compiler version must rebuild, and the loader (which takes ``cc`` from
    the library it loads) must refuse a binary built from other sources."""
    h = hashlib.sha256()
    for rel in HASHED:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(("\0".join([cc or compiler_hash(), *FLAGS])).encode())
    return h.hexdigest()[:16]


def _marker(path: str, marker: bytes) -> str | None:
    try:
        with open(path, "rb") as f:
            blob = f.read()
    except OSError:
        return None
    m = re.search(re.escape(marker) + rb"([0-9a-f]{16}|unknown)\0", blob)
    return m.group(1).decode() if m else None


def library_cc(path: str = None) -> str | None:
    """The compiler identity hash a built library carries (read from the binary, without loading it)."""
    return _marker(path or OUT, CC_MARKER)


def library_id(path: str = OUT) -> str | None:
    """The source id a built library carries (read from the binary, without loading it)."""
    return _marker(path, MARKER)


def needs_build(out: str = OUT) -> bool:
    return library_id(out) != source_id()


def build(force: bool = False, verbose: bool = False) -> str:
    """librp.so. Sources compile in parallel (one hipcc per .hip into build/), then link."""
    out = OUT
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    # one build at a time (two importers racing on the same objects); re-check under the lock
    with open(os.path.join(HERE, "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if force or needs_build(out):
            _compile_and_link(out, verbose)
    return out


def _compile_and_link(out: str, verbose: bool) -> None:
    cc = compiler_hash()
    sid = source_id(cc=cc)
    extra = [f'-DRP_SRC_SHA16="{sid}"', f'-DRP_CC_SHA16="{cc}"']
    odir = os.path.join(HERE, "build", "rel")
    os.makedirs(odir, exist_ok=True)
    objs, procs = [], []
    for src in SRC:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        cmd = [HIPCC, *[f for f in FLAGS if f != "-shared"], *extra, "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        objs.append(obj)
        procs.append(subprocess.Popen(cmd))
    rcs = [p.wait() for p in procs]  # every compile finishes before any failure is raised
    if any(rcs):
        raise subprocess.CalledProcessError(max(rcs), "hipcc")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    if library_id(out + ".tmp") != sid:
        raise RuntimeError(f"{out}.tmp does not carry source id {sid}")
    os.replace(out + ".tmp", out)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
