"""Single-node multi-GPU driver: row shards across GPUs, R broadcast once over RCCL/xGMI.

Replaces the Spark executor layer of the recipe:
  * ``sc.broadcast(local_rnd_mat)`` (code/clustermode/randomProjection.py:104; TorrentBroadcast)
    -> one ``torch.distributed.broadcast`` per device buffer of R's packed image from rank 0 (RCCL
    over xGMI when the backend is ``nccl``); the image is built once, on rank 0 only.
  * ``train.rdd.mapPartitions(...)`` (clustermode:107-110): embarrassingly parallel, no shuffle
    -> every rank projects only its OWN rows: a rank-local host shard (``project_local``), a shard
    already in its HBM (``project_local_device``) or its byte split of a libsvm file
    (``project_libsvm`` / ``libsvm_to_parquet``); no collective inside the row loop.
  * ``monotonically_increasing_id`` (clustermode:72) -> libsvm row ids
    ``((rank << 20) + chunk) << 33 | row``; global row/output offsets of in-memory shards come from
    one tiny all_gather of (rows, nnz) per call.

One process per GPU (``torch.distributed.run``), rank r on ``cuda:LOCAL_RANK``.
"""
from __future__ import annotations

import numpy as np

__all__ = ["plan_shards", "exclusive_offsets", "broadcast_image", "ShardedProjector"]

_META_FIELDS = ("m", "p", "nnz", "layout", "value_type", "magnitude", "block_shift", "n_buffers")
PARTITION_BITS_PER_RANK = 20  # chunk ids per rank in libsvm row ids (partition_base)


def plan_shards(indptr, world: int) -> np.ndarray:
    """Row boundaries (world + 1 entries) of contiguous shards with ~equal nnz (and never an
    inverted range). ``indptr`` is the global CSR row pointer."""
    indptr = np.asarray(indptr, dtype=np.int64)
    n = len(indptr) - 1
    total = int(indptr[-1] - indptr[0])
    if world < 1:
        raise ValueError("world must be >= 1")
    if total == 0:
        bounds = np.linspace(0, n, world + 1).round().astype(np.int64)
    else:
        targets = indptr[0] + (total * np.arange(world + 1, dtype=np.float64) / world)
        bounds = np.searchsorted(indptr, targets, side="left").astype(np.int64)
    bounds[0], bounds[-1] = 0, n
    return np.maximum.accumulate(np.clip(bounds, 0, n))


def exclusive_offsets(counts) -> np.ndarray:
    counts = np.asarray(counts, dtype=np.int64)
    out = np.zeros(counts.size + 1, dtype=np.int64)
    np.cumsum(counts, out=out[1:])
    return out


def broadcast_image(meta, buffers, src: int = 0, group=None):
    """Broadcast R's device image (metadata object + byte buffers) from ``src``.

    ``buffers``: list of uint8 tensors on this rank's device (sized from the metadata, filled
    on ``src``). With the ``nccl`` backend this is RCCL over xGMI; gloo works for CPU tensors."""
    import torch.distributed as dist

    box = [meta]
    dist.broadcast_object_list(box, src=src, group=group)
    for b in buffers:
        dist.broadcast(b, src=src, group=group)
    return box[0]


class ShardedProjector:
    """R resident on every rank's GPU, built on rank 0 and shipped once."""

    def __init__(self, R=None, device: int | None = None, group=None):
        import torch
        import torch.distributed as dist

        from . import _native as nat
        from .projector import Projector

        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.device = torch.cuda.current_device() if device is None else device
        dev = torch.device("cuda", self.device)
        if self.rank == 0:
            if R is None:
                raise ValueError("rank 0 needs R")
            self.projector = Projector(R, device=self.device)
            info = self.projector.info
            meta = {f: getattr(info, f) for f in _META_FIELDS}
            meta["buffer_bytes"] = [int(b) for b in info.buffer_bytes]
            meta["r_index_dtype"] = str(self.projector.r_index_dtype)
            meta["dtype"] = str(self.projector.dtype)
        else:
            meta = None
        if self.world > 1:
            box = [meta]
            dist.broadcast_object_list(box, src=0, group=group)
            meta = box[0]
            bufs = [torch.empty(max(b, 1), dtype=torch.uint8, device=dev)
                    for b in meta["buffer_bytes"][:meta["n_buffers"]]]
            if self.rank == 0:
                self.projector.export_image([b.data_ptr() for b in bufs])
            for b in bufs:
                dist.broadcast(b, src=0, group=group)
            torch.cuda.synchronize(dev)
            if self.rank != 0:
                info = nat.ProjectorInfo()
                for f in _META_FIELDS:
                    setattr(info, f, meta[f])
                for i, b in enumerate(meta["buffer_bytes"]):
                    info.buffer_bytes[i] = b
                self.projector = Projector.from_image(info, [b.data_ptr() for b in bufs], device=self.device,
                                                      r_index_dtype=meta["r_index_dtype"], dtype=meta["dtype"])
            del bufs
        self.meta = meta
        self.group = group

    # ---- rank-local work: every rank projects only its own rows (clustermode:107-110)
    def _gather_counts(self, *vals):
        """all_gather of a few int64 per rank -> (world, len(vals)) array (the only collective,
        once per call, outside any row loop)."""
        import torch
        import torch.distributed as dist

        t = torch.tensor([list(vals)], dtype=torch.int64)
        if self.world == 1:
            return t.numpy()
        if dist.get_backend(self.group) == "nccl":
            t = t.cuda(self.device)
        allc = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(allc, t, group=self.group)
        return np.concatenate([x.cpu().numpy() for x in allc])

    def project_local(self, A_local, order: str = "scipy"):
        """Project this rank's own shard (host CSR, any rows: the shards of ranks 0..world-1 are
        consecutive row ranges of the global matrix). Returns ``(row_offset, nnz_offset, C_local)``:
        the global index of the shard's first row and first output entry, and ``A_local @ R``."""
        import scipy.sparse as sp

        A_local = sp.csr_matrix(A_local)
        C = self.projector.matmul(A_local, order=order)
        cnt = self._gather_counts(A_local.shape[0], C.nnz)
        rows, nnz = exclusive_offsets(cnt[:, 0]), exclusive_offsets(cnt[:, 1])
        return int(rows[self.rank]), int(nnz[self.rank]), C

    def project_local_device(self, Ap, Aj, Ax, order: str = "scipy", stream=None):
        """Project a rank-local shard already in this rank's HBM (torch tensors; ``Ap`` may start at
        any value). Returns ``(row_offset, nnz_offset, Cp, Cj, Cx, nnz)`` with device outputs
        sized exactly (int64 indptr when nnz needs it)."""
        import torch

        from . import _native as nat

        dev = torch.device("cuda", self.device)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        n = Ap.numel() - 1
        nnz_a = int(Ap[-1].item()) - int(Ap[0].item()) if n > 0 else 0
        P = self.projector
        ws = torch.empty(max(P.workspace_bytes(n, nnz_a), 1), dtype=torch.uint8, device=dev)
        cap = int(1.02 * nnz_a * P.nnz / max(P.m, 1)) + 65536
        for _ in range(2):
            Cp = torch.empty(n + 1, dtype=torch.int64 if cap >= 2**31 else torch.int32, device=dev)
            Cj = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
            Cx = torch.empty(max(cap, 1), dtype=Ax.dtype, device=dev)
            try:
                k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=order, stream=stream, workspace=ws, nnz_a=nnz_a)
                break
            except nat.RPError as e:
                if e.code != nat.RP_ERR_CAPACITY:
                    raise
                cap = e.nnz
        del ws
        cnt = self._gather_counts(n, k)
        rows, nnz = exclusive_offsets(cnt[:, 0]), exclusive_offsets(cnt[:, 1])
        return int(rows[self.rank]), int(nnz[self.rank]), Cp, Cj[:k], Cx[:k], k

    def byte_range(self, path: str):
        """This rank's split of a text file: an equal share of its bytes (lines are assigned by
        where they start, libsvm.split_range)."""
        import os

        size = os.path.getsize(path)
        return size * self.rank // self.world, size * (self.rank + 1) // self.world

    def partition_base(self) -> int:
        """First partition id of this rank's chunks: ``rank << 20`` (2^20 chunks per rank), so row
        ids ``(partition << 33) + row`` are unique and increasing in file order across ranks, as
        Spark's monotonically_increasing_id (clustermode:72) guarantees (unique, increasing, not
        consecutive)."""
        return self.rank << PARTITION_BITS_PER_RANK

    def project_libsvm(self, path: str, chunk_bytes: int = None, order: str = "sorted"):
        """This rank's split of a libsvm file -> GPU parse -> projection, per chunk:
        ``(ids, labels, C)`` (libsvm.project_libsvm). No rank reads another rank's bytes."""
        from . import libsvm

        kw = {} if chunk_bytes is None else {"chunk_bytes": chunk_bytes}
        return libsvm.project_libsvm(path, self.projector, order=order, byte_range=self.byte_range(path),
                                     partition_base=self.partition_base(), **kw)

    def libsvm_to_parquet(self, path: str, out_dir: str, chunk_bytes: int = None):
        """The recipe end to end on this rank's split: Parquet part files in ``out_dir``
        (clustermode:71-80,107-113). Returns this rank's part paths."""
        from . import libsvm

        kw = {} if chunk_bytes is None else {"chunk_bytes": chunk_bytes}
        return libsvm.libsvm_to_parquet(path, self.projector, out_dir, byte_range=self.byte_range(path),
                                        partition_base=self.partition_base(), **kw)

    def project_partition(self, A, order: str = "scipy"):
        """Convenience for a GLOBAL host CSR every rank holds: projects this rank's nnz-balanced
        row range of it (``plan_shards``) through ``project_local``."""
        import scipy.sparse as sp

        A = sp.csr_matrix(A)
        bounds = plan_shards(A.indptr, self.world)
        r0, r1 = int(bounds[self.rank]), int(bounds[self.rank + 1])
        return self.project_local(A[r0:r1], order=order)
