"""Single-node multi-GPU driver: row shards across GPUs, R broadcast once over RCCL/xGMI.

Replaces the Spark executor layer of the recipe:
  * ``sc.broadcast(local_rnd_mat)`` (code/clustermode/randomProjection.py:104; TorrentBroadcast)
    -> one ``torch.distributed.broadcast`` per device buffer of R's packed image from rank 0 (RCCL
    over xGMI when the backend is ``nccl``); the image is built once, on rank 0 only.
  * ``train.rdd.mapPartitions(...)`` (clustermode:107-110): embarrassingly parallel, no shuffle
    -> contiguous row shards balanced by nnz, one per rank, no collective inside the row loop.
  * ``monotonically_increasing_id`` / global row numbering (clustermode:72) -> each rank knows its
    global row offset; global output offsets come from one tiny all_gather of shard nnz.

One process per GPU (``torch.distributed.run``), rank r on ``cuda:LOCAL_RANK``.
"""
from __future__ import annotations

import numpy as np

__all__ = ["plan_shards", "exclusive_offsets", "broadcast_image", "ShardedProjector"]

_META_FIELDS = ("m", "p", "nnz", "layout", "value_type", "magnitude", "block_shift", "n_buffers")


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

    def project_partition(self, A, order: str = "scipy"):
        """Project this rank's shard of the global CSR ``A`` (host). Returns
        ``(row_offset, nnz_offset, C_local)``: the shard's first global row, the global position of
        its first output entry, and its rows of ``A @ R`` (scipy CSR)."""
        import scipy.sparse as sp
        import torch
        import torch.distributed as dist

        A = sp.csr_matrix(A)
        bounds = plan_shards(A.indptr, self.world)
        r0, r1 = int(bounds[self.rank]), int(bounds[self.rank + 1])
        C = self.projector.matmul(A[r0:r1], order=order)
        counts = np.array([C.nnz], dtype=np.int64)
        if self.world > 1:
            t = torch.tensor(counts, dtype=torch.int64)
            if dist.get_backend(self.group) == "nccl":
                t = t.cuda(self.device)
            allc = [torch.zeros_like(t) for _ in range(self.world)]
            dist.all_gather(allc, t, group=self.group)
            counts = np.array([int(x.item()) for x in allc], dtype=np.int64)
        offs = exclusive_offsets(counts)
        return r0, int(offs[self.rank]), C
