"""(Historical, round 1: it sets environment knobs librp no longer reads — rp_projector_set_option
replaced them in round 3; kept as the record of DESIGN.md §3d's measurement.)
Feasibility probe for a hybrid direct + staged step (configs[1] shape), measurement only.

(1) Direct tile kernel alone with fewer tiles resident per CU (RP_DEBUG_LDS_PAD inflates its LDS):
    does the random-line request rate still saturate with a fraction of the slots?
(2) Rows split in two halves: the direct kernel on one, the staged pipeline on the other, run one
    after the other on one stream vs concurrently on two streams.

    python scripts/probes/hybrid_probe.py [--rows N] [--out gpurun_out/hybrid_probe.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=119_705_032)
    ap.add_argument("--split", type=float, default=0.5, help="fraction of rows on the direct kernel")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "hybrid_probe.json"))
    args = ap.parse_args()

    import torch

    torch.cuda.set_device(0)
    from randomprojection_amd import Projector, srp_matrix as sm, synth

    dev = torch.device("cuda", 0)
    R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
    Ap, Aj, Ax = synth.kdd_rows_device(args.rows, sm.KDD_M, seed=2012)
    Ap = Ap.to(torch.int64)
    torch.cuda.synchronize()
    n = args.rows
    res = {"rows": n}

    def outputs(rows, nnz):
        cap = int(1.05 * nnz * R.nnz / R.shape[0]) + 65536
        return (torch.empty(rows + 1, dtype=torch.int64, device=dev), torch.empty(cap, dtype=torch.int32, device=dev),
                torch.empty(cap, dtype=torch.float32, device=dev))

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    # (1) residency sweep, whole matrix, direct
    P = Projector(R)
    P.set_staging("off")
    nnz = int(Aj.numel())
    ws = torch.empty(P.workspace_bytes(n, nnz), dtype=torch.uint8, device=dev)
    Cp, Cj, Cx = outputs(n, nnz)
    st = torch.cuda.current_stream(dev).cuda_stream
    sweep = {}
    for pad in (0, 26000, 52000, 78000, 130000):
        os.environ["RP_DEBUG_LDS_PAD"] = str(pad)
        ms = timed(lambda: P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, stream=st, workspace=ws, nnz_a=nnz, sync=False))
        sweep[str(pad)] = ms
        print(f"pad {pad}: {ms:.2f} ms", flush=True)
    os.environ.pop("RP_DEBUG_LDS_PAD")
    res["direct_ms_by_lds_pad"] = sweep
    del ws, Cp, Cj, Cx
    torch.cuda.empty_cache()

    # (2) halves: direct on rows [0, h), staged on rows [h, n)
    h = int(n * args.split)
    Ap1, Ap2 = Ap[:h + 1], Ap[h:]
    nnz1 = int(Ap[h].item())
    nnz2 = nnz - nnz1
    P1 = Projector(R)
    P1.set_staging("off")
    P2 = Projector(R)
    P2.set_staging("on")
    ws1 = torch.empty(P1.workspace_bytes(h, nnz1), dtype=torch.uint8, device=dev)
    ws2 = torch.empty(P2.workspace_bytes(n - h, nnz2), dtype=torch.uint8, device=dev)
    o1, o2 = outputs(h, nnz1), outputs(n - h, nnz2)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def run1(stream):
        P1.project_device(Ap1, Aj, Ax, *o1, stream=stream.cuda_stream, workspace=ws1, nnz_a=nnz1, sync=False)

    def run2(stream):
        P2.project_device(Ap2, Aj, Ax, *o2, stream=stream.cuda_stream, workspace=ws2, nnz_a=nnz2, sync=False)

    res["split"] = args.split
    res["half_direct_ms"] = timed(lambda: run1(s1))
    res["half_staged_ms"] = timed(lambda: run2(s1))
    res["sequential_ms"] = timed(lambda: (run1(s1), run2(s1)))
    res["concurrent_ms"] = timed(lambda: (run1(s1), run2(s2)))
    for pad in (52000, 78000):
        os.environ["RP_DEBUG_LDS_PAD"] = str(pad)
        res[f"concurrent_direct_pad{pad}_ms"] = timed(lambda: (run1(s1), run2(s2)))
    os.environ.pop("RP_DEBUG_LDS_PAD")
    print(json.dumps(res, indent=1), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
