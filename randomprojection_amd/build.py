"""Build librp.so (HIP, gfx950) in-tree with hipcc. No CUDA, no hipify, no multi-target build."""
from __future__ import annotations

import fcntl
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(HERE, "csrc", n) for n in ("rp_spgemm.hip", "rp_libsvm.hip", "rp_dense.hip")]
OUT = os.path.join(HERE, "librp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    # scipy's csr_matmat rounds the multiply and the add separately: never contract to FMA
    "-ffp-contract=off", "-fno-fast-math", "-Wall",
]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SRC + [os.path.join(HERE, "..", "include", "rp.h"), os.path.join(HERE, "csrc", "rp_common.h"),
                  os.path.join(HERE, "csrc", "rp_pow5.h")]
    return any(os.path.getmtime(s) > t for s in deps)


DIAG_OUT = os.path.join(HERE, "librp_diag.so")


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    """librp.so; ``diag=True`` builds librp_diag.so instead (in-kernel stage stamps, -DRP_STAMPS),
    used only by scripts/stage_stamps.py, never by the package. Sources compile in parallel (one
    hipcc per .hip into build/), then link."""
    out = DIAG_OUT if diag else OUT
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    # one build at a time (two importers racing on the same objects); re-check under the lock
    with open(os.path.join(HERE, "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if force or diag or needs_build():
            _compile_and_link(out, diag, verbose)
    return out


def _compile_and_link(out: str, diag: bool, verbose: bool) -> None:
    extra = ["-DRP_STAMPS"] if diag else []
    odir = os.path.join(HERE, "build", "diag" if diag else "rel")
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
    os.replace(out + ".tmp", out)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
