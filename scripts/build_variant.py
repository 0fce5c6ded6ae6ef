"""Build librp from a source variant into another file (A/B measurements: bench.py --lib <file>):
    [VARIANT_FLAGS="-DNAME=value ..."] python scripts/build_variant.py <variant.hip> <out.so>
The variant replaces csrc/rp_spgemm.hip; rp_libsvm.hip is shared. Its build id is the sha256
prefix of the variant file and the extra flags (so a line measured on it never carries the
package's id)."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from randomprojection_amd.build import FLAGS, HIPCC, SRC  # noqa: E402

src = [sys.argv[1]] + [s for s in SRC if not s.endswith("rp_spgemm.hip")]
if "0d702fa" in open(sys.argv[1]).read(20000) or os.environ.get("NO_DENSE"):
    src = [s for s in src if not s.endswith("rp_dense.hip")]
inc = ["-I", os.path.join(ROOT, "randomprojection_amd", "csrc"), "-I", os.path.join(ROOT, "include")]
extra = os.environ.get("VARIANT_FLAGS", "").split()
vid = hashlib.sha256(open(sys.argv[1], "rb").read() + " ".join(extra).encode()).hexdigest()[:16]
subprocess.run([HIPCC, *FLAGS, *inc, *extra, f'-DRP_SRC_SHA16="{vid}"', "-o", sys.argv[2], *src], check=True)
print(sys.argv[2])
