"""Dense Gaussian projection benchmark (BASELINE.json configs[4]: 10M x 16384 -> 1024, fp32/bf16).

Two labelled measurements, one JSON line each:
  * "resident": one GEMM of a `--chunk`-row block of synthetic N(0,1) X already in HBM by the
    1024 x 16384 components (sklearn-identical normal draws, random_state=123) — librp's
    hand-written MFMA kernel (rp_dense_project_device) and, for comparison, torch's matmul
    (hipBLASLt); MFMA TFLOP/s against the dense peak (f32 157.3 TF, bf16 2.5 PF).
  * "stream": the whole pass as it must run (X = 655 GB f32 / 328 GB bf16 does not fit in HBM):
    X chunks in page-locked host memory (a ring of `--ring` distinct chunks, cycled), uploaded on a
    copy stream while the previous chunk's GEMM runs on the compute stream, Y downloaded into
    page-locked host memory; rows/s over `--stream-chunks` chunks, and the full 10M-row pass time
    it implies (PCIe-bound: ~64 KB/row f32, ~32 KB/row bf16 in).

    python scripts/bench_dense.py [--compute fp32|bf16] [--chunk 131072] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_TF = {"fp32": 157.3, "bf16": 2500.0, "fp64": 78.6}  # MI355X dense peaks (fp64 matrix = vector rate)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compute", choices=["fp32", "bf16", "fp64"], default="fp32")
    ap.add_argument("--chunk", type=int, default=131072)
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--p", type=int, default=1024)
    ap.add_argument("--rows-total", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stream-chunk", type=int, default=32768)
    ap.add_argument("--stream-chunks", type=int, default=24)
    ap.add_argument("--ring", type=int, default=3)
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--variant", type=int, default=-1, help="librp dense tile variant (rp_dense_project_device variant, per call)")
    ap.add_argument("--lib", default=None, help="another librp build (A/B measurements; its id is reported)")
    args = ap.parse_args()

    import torch

    from randomprojection_amd.gaussian import dense_project_device
    from randomprojection_amd.srp_matrix import gaussian_random_matrix

    from randomprojection_amd import _native as nat

    nat.load(args.lib)
    torch.cuda.set_device(0)
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[args.compute]
    C = torch.as_tensor(gaussian_random_matrix(args.p, args.m, random_state=123).astype("float32"), device="cuda")
    C = C.to(dt)
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn(args.chunk, args.m, device="cuda", generator=g).to(dt)
    out = torch.empty(args.chunk, args.p, device="cuda", dtype=torch.float64 if dt == torch.float64 else torch.float32)
    flop = 2.0 * args.chunk * args.m * args.p

    def torch_mm():
        if dt == torch.bfloat16:
            torch.mm(X, C.t(), out_dtype=torch.float32, out=out)
        else:
            torch.mm(X, C.t(), out=out)

    def ours():
        dense_project_device(X, C, out=out, compute=args.compute, variant=args.variant)

    res = {}
    for name, fn in (("librp_mfma", ours), ("torch_hipblaslt", torch_mm)):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        res[name] = {"ms": ms, "tflops": flop / (ms * 1e-3) / 1e12}
    # accuracy: both GEMMs against an fp64 product of the SAME (dtype-rounded) operands, on 512 rows
    # spread over the block (two f32-accumulating GEMMs differ only in summation order)
    rows = torch.arange(0, args.chunk, max(1, args.chunk // 512), device="cuda")[:512]
    ref = X[rows].double() @ C.double().t()
    dense_project_device(X, C, out=out, compute=args.compute, variant=args.variant)
    rel_ours = float((out[rows].double() - ref).norm() / ref.norm())
    torch_mm()
    rel_torch = float((out[rows].double() - ref).norm() / ref.norm())
    ms = res["librp_mfma"]["ms"]
    tf = res["librp_mfma"]["tflops"]
    print(json.dumps({
        "metric": "rows/sec projected, dense Gaussian 16384 -> 1024 (configs[4]), X resident in HBM",
        "value": args.chunk / (ms * 1e-3), "unit": "rows/s", "n_gpus": 1, "steps": args.steps,
        "ms_per_step": ms, "dtype": args.compute, "data": "synthetic N(0,1) X, sklearn-identical components",
        "config": {"workload": f"configs[4]: one {args.chunk} x {args.m} block of X in HBM -> {args.p}",
                   "boundary": "device"},
        "roofline": {"bound": "mfma", "achieved": tf, "peak": PEAK_TF[args.compute], "unit": "TFLOP/s",
                     "frac": tf / PEAK_TF[args.compute], "kernel": "rp_dense_project_device (csrc/rp_dense.hip)"},
        "library_comparison": res, "variant": args.variant,
        "rel_err_vs_fp64_same_operands": {"librp": rel_ours, "torch": rel_torch},
    }), flush=True)
    if args.no_stream:
        return
    del X, out
    torch.cuda.empty_cache()
    # ---- stream: pinned host X ring -> H2D on a copy stream, GEMM on the compute stream, Y -> host
    cs, ks = torch.cuda.Stream(), torch.cuda.Stream()
    n = args.stream_chunk
    hx = [torch.randn(n, args.m, generator=torch.Generator().manual_seed(k)).to(dt).pin_memory()
          for k in range(args.ring)]
    hy = [torch.empty(n, args.p, dtype=torch.float32).pin_memory() for _ in range(2)]
    dx = [torch.empty(n, args.m, dtype=dt, device="cuda") for _ in range(2)]
    dy = [torch.empty(n, args.p, dtype=torch.float32, device="cuda") for _ in range(2)]
    up = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in range(2)]

    def run(chunks):
        for k in range(chunks):
            b = k & 1
            with torch.cuda.stream(cs):
                if k >= 2:
                    cs.wait_event(done[b])  # the GEMM that read dx[b] two chunks ago is finished
                dx[b].copy_(hx[k % args.ring], non_blocking=True)
                up[b].record(cs)
            with torch.cuda.stream(ks):
                ks.wait_event(up[b])
                dense_project_device(dx[b], C, out=dy[b], compute=args.compute, stream=ks.cuda_stream)
                hy[b].copy_(dy[b], non_blocking=True)
                done[b].record(ks)
        torch.cuda.synchronize()

    run(4)
    t0 = time.perf_counter()
    run(args.stream_chunks)
    wall = time.perf_counter() - t0
    rows_s = args.stream_chunks * n / wall
    h2d = args.stream_chunks * n * args.m * (2 if dt == torch.bfloat16 else 4)
    print(json.dumps({
        "metric": "rows/sec projected, dense Gaussian 16384 -> 1024 (configs[4]), X streamed from host",
        "value": rows_s, "unit": "rows/s", "n_gpus": 1, "dtype": args.compute,
        "data": "synthetic N(0,1) X in page-locked host memory (a ring of distinct chunks)",
        "config": {"workload": f"configs[4] streamed: {n}-row chunks, H2D overlapped with the GEMM, Y to host",
                   "boundary": "host", "chunks": args.stream_chunks},
        "pcie": {"h2d_GBps": h2d / wall / 1e9, "link_peak_GBps_per_direction": 63.0},
        "full_projection_s": args.rows_total / rows_s,
    }), flush=True)


if __name__ == "__main__":
    main()
