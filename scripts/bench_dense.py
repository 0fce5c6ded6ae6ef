"""Dense Gaussian projection benchmark (BASELINE.json configs[4]: 10M x 16384 -> 1024, fp32/bf16).

X does not fit in HBM at full size (655 GB f32), so it is streamed: one step = one GEMM of a
`--chunk`-row block of synthetic N(0,1) X (generated in HBM once) by the 1024 x 16384 components
(sklearn-identical numpy normal draws, random_state=123); throughput in rows/s and MFMA TFLOP/s
against the dense peak (f32 157.3 TF, bf16 2.5 PF; MI355X_MICROARCH.md). Prints one JSON line.

    python scripts/bench_dense.py [--compute fp32|bf16] [--chunk 131072] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_TF = {"fp32": 157.3, "bf16": 2500.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compute", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--chunk", type=int, default=131072)
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--p", type=int, default=1024)
    ap.add_argument("--rows-total", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()

    import torch

    from randomprojection_amd.gaussian import dense_project_device
    from randomprojection_amd.srp_matrix import gaussian_random_matrix

    torch.cuda.set_device(0)
    C = torch.as_tensor(gaussian_random_matrix(args.p, args.m, random_state=123).astype("float32"), device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn(args.chunk, args.m, device="cuda", generator=g)
    if args.compute == "bf16":
        X = X.to(torch.bfloat16)
        C = C.to(torch.bfloat16)
    out = torch.empty(args.chunk, args.p, device="cuda", dtype=torch.float32)
    for _ in range(args.warmup):
        dense_project_device(X, C, out=out, compute=args.compute)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        dense_project_device(X, C, out=out, compute=args.compute)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    ms = e0.elapsed_time(e1) / args.steps
    flop = 2.0 * args.chunk * args.m * args.p
    tf = flop / (ms * 1e-3) / 1e12
    print(json.dumps({
        "metric": "rows/sec projected, dense Gaussian 16384 -> 1024 (configs[4])",
        "value": args.chunk / wall, "unit": "rows/s", "n_gpus": 1, "steps": args.steps,
        "ms_per_step": wall * 1e3, "dtype": args.compute, "data": "synthetic N(0,1) X, sklearn-identical components",
        "config": {"workload": f"configs[4] streamed: {args.chunk}-row chunks of {args.rows_total} x {args.m} -> {args.p}"},
        "roofline": {"bound": "mfma", "achieved": tf, "peak": PEAK_TF[args.compute], "unit": "TFLOP/s",
                     "frac": tf / PEAK_TF[args.compute]},
        "full_projection_s": args.rows_total / (args.chunk / wall),
    }))


if __name__ == "__main__":
    main()
