"""Probe variant of librp (timing only, never the product): the staged gather kernel without its W32
lookups (D = the feature word itself), so a profile of it shows what the S/D streams alone cost and
which of the kernel's L2 requests are the W32 lookups' (roofline.l2_hit_rate_r_gathers).
    python scripts/probes/make_gather_probe.py variants/gather_now32.hip
    python scripts/build_variant.py variants/gather_now32.hip variants/gather_now32.so"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "randomprojection_amd", "csrc", "rp_spgemm.hip")).read()
old = "w[u] = __builtin_amdgcn_raw_buffer_load_b32(wr, hit ? col * 4u : kOob, 0, 0);"
assert src.count(old) == 1, "gather kernel changed: update the probe"
open(sys.argv[1], "w").write(src.replace(old, "w[u] = hit ? col : 0u;"))
