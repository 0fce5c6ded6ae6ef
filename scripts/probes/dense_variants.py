"""Probe: librp dense MFMA GEMM tile variants (rp_dense_project_device variant, per call) — correctness on a ragged shape
against an fp64 product, then TFLOP/s on the configs[4] block (131072 x 16384 -> 1024)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from randomprojection_amd.gaussian import dense_project_device  # noqa: E402

variants = [int(v) for v in sys.argv[1].split(",")]
torch.cuda.set_device(0)
rng = np.random.default_rng(0)
Xs = torch.as_tensor(rng.standard_normal((700, 4096)).astype(np.float32), device="cuda")
Cs = torch.as_tensor(rng.normal(0, 1 / 32, (300, 4096)).astype(np.float32), device="cuda")
g = torch.Generator(device="cuda").manual_seed(5)
Xb = torch.randn(131072, 16384, device="cuda", generator=g)
Cb = torch.randn(1024, 16384, device="cuda", generator=g) / 32
res = {}
for comp in ("bf16", "fp32"):
    dt = torch.bfloat16 if comp == "bf16" else torch.float32
    X, C = Xb.to(dt), Cb.to(dt)
    out = torch.empty(131072, 1024, device="cuda")
    ref = Xs.to(dt).double().cpu().numpy() @ Cs.to(dt).double().cpu().numpy().T
    for v in variants:
        Y = dense_project_device(Xs, Cs, compute=comp, variant=v).cpu().numpy()
        rel = float(np.linalg.norm(Y - ref) / np.linalg.norm(ref))
        for _ in range(2):
            dense_project_device(X, C, out=out, compute=comp, variant=v)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dense_project_device(X, C, out=out, compute=comp, variant=v)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        tf = 2 * 131072 * 16384 * 1024 / (ms * 1e-3) / 1e12
        res[f"{comp}_v{v}"] = {"ms": round(ms, 3), "tflops": round(tf, 1), "rel_err": rel}
        print(comp, v, res[f"{comp}_v{v}"], flush=True)
    del X, C
print(json.dumps(res))
