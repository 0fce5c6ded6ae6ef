"""randomprojection_amd — MI355X-native projection step of afcarl/RandomProjection.

The hot path is ``X_partition @ R`` (code/clustermode/randomProjection.py:46): a row-split
Gustavson SpGEMM written in HIP for gfx950 (randomprojection_amd/csrc/rp_spgemm.hip) behind the
C-ABI of include/rp.h, bit-identical to scipy's csr_matmat. Python drop-ins mirror the reference's
interfaces:

* ``random_project_mappartitions_function`` / ``random_project_map_function`` (partition.py)
* ``SparseRandomProjection`` with GPU ``transform`` (random_projection.py)
* ``Projector`` — R resident in HBM, ``matmul(A)`` == scipy ``A @ R`` (projector.py)
* ``srp_matrix.sparse_random_matrix`` — sklearn's R generator, bit-identical and vectorised
* ``driver`` — single-node multi-GPU sharding with one RCCL broadcast of R
"""
from . import srp_matrix
from ._native import NativeUnavailable, RPError
from .linalg import SparseVector, Vectors
from .partition import random_project_map_function, random_project_mappartitions_function
from .projector import Projector, get_projector
from .srp_matrix import johnson_lindenstrauss_min_dim

__all__ = [
    "Projector", "get_projector", "random_project_mappartitions_function",
    "random_project_map_function", "SparseRandomProjection", "SparseVector", "Vectors",
    "srp_matrix", "johnson_lindenstrauss_min_dim", "NativeUnavailable", "RPError",
]
__version__ = "0.1.0"


def __getattr__(name):  # sklearn is imported lazily (the partition path does not need it)
    if name == "SparseRandomProjection":
        from .random_projection import SparseRandomProjection

        return SparseRandomProjection
    raise AttributeError(name)
