"""Probe: configs[1] rows projected as K row partitions (the recipe's mapPartitions unit), each its
own rp_project_device call with its own workspace and CSR output, issued round-robin on S HIP
streams, so one partition's deferred-tile copy can overlap another partition's gather-bound main
kernel. Prints ms per pass over all rows for each (K, S); checks every partition's nnz adds up to
the single-call result.

    python scripts/probes/partition_streams_probe.py [--steps 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=119_705_032)
    ap.add_argument("--m", type=int, default=54_686_452)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--dist", default="uniform")
    args = ap.parse_args()
    import torch

    from randomprojection_amd import Projector, srp_matrix as sm, synth

    dev = torch.device("cuda", 0)
    P = Projector(sm.projection_operand(sm.sparse_random_matrix(4096, args.m, random_state=123)))
    Ap, Aj, Ax = synth.kdd_rows_device(args.rows, args.m, seed=2012, dist=args.dist, device=0)
    torch.cuda.synchronize()
    ap_host = Ap.cpu()
    out = {"rows": args.rows, "dist": args.dist, "runs": []}
    for K, S in ((1, 1), (2, 2), (4, 2), (8, 2), (4, 4)):
        bounds = [args.rows * k // K for k in range(K + 1)]
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        parts = []
        for k in range(K):
            r0, r1 = bounds[k], bounds[k + 1]
            n = r1 - r0
            nnz = int(ap_host[r1] - ap_host[r0])
            cap = int(1.05 * nnz * P.nnz / P.m) + 65536
            parts.append(dict(
                Ap=Ap[r0:r1 + 1], n=n, nnz=nnz,
                ws=torch.empty(P.workspace_bytes(n, nnz), dtype=torch.uint8, device=dev),
                Cp=torch.empty(n + 1, dtype=torch.int32, device=dev),
                Cj=torch.empty(cap, dtype=torch.int32, device=dev),
                Cx=torch.empty(cap, dtype=torch.float32, device=dev)))

        def one_pass(sync=False):
            tot = 0
            for k, q in enumerate(parts):
                st = streams[k % S]
                tot += P.project_device(q["Ap"], Aj, Ax, q["Cp"], q["Cj"], q["Cx"], stream=st.cuda_stream,
                                        workspace=q["ws"], nnz_a=q["nnz"], sync=sync) or 0
            return tot

        torch.cuda.synchronize()
        nnz_c = one_pass(sync=True)
        for _ in range(2):
            one_pass()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_pass()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        run = {"partitions": K, "streams": S, "ms_per_pass": ms, "rows_per_s": args.rows / ms * 1e3, "nnz_c": nnz_c}
        out["runs"].append(run)
        print(json.dumps(run), flush=True)
        del parts
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
