"""One rank of tests/test_gpu_dist.py (launched as a child process with RANK/WORLD_SIZE/MASTER_*):
every rank on cuda:0 over gloo (RCCL needs one GPU per rank; this box has one), R built on rank 0
only and shipped by ShardedProjector's broadcast, each rank projecting only its own rows."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import scipy.sparse as sp
    import torch
    import torch.distributed as dist

    from randomprojection_amd import srp_matrix as sm
    from randomprojection_amd.driver import ShardedProjector, plan_shards

    out_dir, text_path = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    m, p = 300_000, 256
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123)) if rank == 0 else None
    S = ShardedProjector(R, device=0)
    # the global matrix exists only to cut this rank's own rows out of it (a rank's local data)
    rng = np.random.default_rng(5)
    n = 40_000
    k = 1 + rng.poisson(10, n)
    k[::101] = 0
    ip = np.concatenate([[0], np.cumsum(k)])
    A = sp.csr_matrix((rng.standard_normal(ip[-1]).astype(np.float32), rng.integers(0, m, ip[-1]).astype(np.int32),
                       ip), shape=(n, m))
    A.sum_duplicates()
    b = plan_shards(A.indptr, world)
    r0, r1 = int(b[rank]), int(b[rank + 1])
    row_off, nnz_off, C = S.project_local(A[r0:r1])
    # the same rows already in HBM, indptr not starting at 0, entries of the whole matrix
    dev = torch.device("cuda", 0)
    Ap = torch.as_tensor(A.indptr[r0:r1 + 1].astype(np.int64), device=dev)
    Aj = torch.as_tensor(A.indices, device=dev)
    Ax = torch.as_tensor(A.data, device=dev)
    d_row, d_nnz, Cp, Cj, Cx, kk = S.project_local_device(Ap, Aj, Ax)
    parts = S.libsvm_to_parquet(text_path, os.path.join(out_dir, "parquet"), chunk_bytes=1 << 14)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), row_off=row_off, nnz_off=nnz_off, indptr=C.indptr,
             indices=C.indices, data=C.data, d_row=d_row, d_nnz=d_nnz, d_indptr=Cp.cpu().numpy(),
             d_indices=Cj.cpu().numpy(), d_data=Cx.cpu().numpy(), parts=np.array(parts), A_indptr=A.indptr,
             A_indices=A.indices, A_data=A.data, byte_range=np.array(S.byte_range(text_path)))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
