"""Where does a tile's time go? Runs the diagnostic build (librp_diag.so, -DRP_STAMPS) on synthetic
KDD-shaped rows and prints per-stage durations from in-kernel s_memrealtime stamps (100 MHz).
Diagnostic only: stamps perturb timing; read the SHARES, not the absolute kernel time.

    python scripts/stage_stamps.py [--rows N] [--dist uniform|powerlaw]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--dist", default="uniform")
    ap.add_argument("--staging", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--p", type=int, default=4096)
    ap.add_argument("--mean-extra", type=float, default=10.0)
    ap.add_argument("--rpt", type=int, default=256, help="rows per tile the launch will use")
    ap.add_argument("--lpr", action="store_true", help="stamps of the row-lane pipeline (stage names)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "stamps.json"))
    args = ap.parse_args()

    import torch

    torch.cuda.set_device(0)   # initialise torch's HIP context before librp touches the device
    from randomprojection_amd import _native as nat
    lib = nat.load(os.path.join(ROOT, "randomprojection_amd", "librp_diag.so"))
    lib.rp_debug_stamps.argtypes = [ctypes.c_void_p]
    from randomprojection_amd import Projector, srp_matrix as sm, synth

    m = args.m or sm.KDD_M
    R = sm.projection_operand(sm.sparse_random_matrix(args.p, m, random_state=123))
    P = Projector(R)
    P.set_staging(args.staging)
    Ap, Aj, Ax = synth.kdd_rows_device(args.rows, m, seed=7, dist=args.dist, mean_extra=args.mean_extra)
    n_tiles = (args.rows + args.rpt - 1) // args.rpt
    stamps = torch.zeros(n_tiles * 8, dtype=torch.int64, device="cuda")
    cap = int(1.3 * Aj.numel() * P.nnz / P.m) + 1024
    Cp = torch.empty(args.rows + 1, dtype=torch.int32, device="cuda")
    Cj = torch.empty(cap, dtype=torch.int32, device="cuda")
    Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
    nat.check(lib.rp_debug_stamps(ctypes.c_void_p(0)))
    P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, nnz_a=Aj.numel())          # warm, no stamps
    nat.check(lib.rp_debug_stamps(ctypes.c_void_p(stamps.data_ptr())))
    P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, nnz_a=Aj.numel())
    torch.cuda.synchronize()
    st = stamps.view(n_tiles, 8).cpu().numpy().astype(np.int64)
    t0 = st[:, 0].min()
    names = ["gather-or-staged-read(1a)", "scan(1b)", "products(1c)", "accumulate(2)", "scan+lookback(3a)", "write(3b)"]
    if args.lpr:
        names = ["descs(wait round2)", "barrier+round1-issue", "flatpass", "side-fill+next-runs(3 barriers)",
                 "rows+exact+slot-store", "-"]
    res = {"tiles": int(n_tiles), "heavy_tiles": int((st[:, 7] > 0).sum())}
    ok = st[:, 6] > 0
    for k, nm in enumerate(names):
        d = (st[ok, k + 1] - st[ok, k]) * 10.0 / 1000.0  # 100 MHz ticks -> us
        res[nm] = {"median_us": float(np.median(d)), "p90_us": float(np.percentile(d, 90)), "mean_us": float(d.mean())}
    life = (st[ok, 6] - st[ok, 0]) * 10.0 / 1000.0
    res["tile_life_us"] = {"median": float(np.median(life)), "p90": float(np.percentile(life, 90))}
    span = (st[ok, 6].max() - t0) * 10.0 / 1e6
    res["kernel_span_ms"] = float(span)
    # mean concurrency = sum of lifetimes / span
    res["mean_tiles_in_flight"] = float(life.sum() / 1000.0 / span)
    print(json.dumps(res, indent=1))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
