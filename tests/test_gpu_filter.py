"""Filtered tile pipeline (RP_OPT_FILTER): a streaming pass drops the A entries whose
R row is empty, then the tile kernel runs on what is left. Bit for bit equal to the oracle's
restatement of scipy's csr_matmat (and so to the unfiltered tile pipeline): configs[3]-shaped rows
over a 10M-feature R (27% of its rows nonempty), f32/f64, both orders, uniform and power-law
columns, empty rows, rows whose every feature has an empty R row, filter units longer than one
round (rows of thousands of entries, which also take the exact slow path), several row chunks,
deferral forced and forbidden, and the unfiltered fallback."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import smmp
from randomprojection_amd import Projector, srp_matrix as sm
from test_gpu_parity import assert_same_csr, kdd_like, oracle_product

pytestmark = pytest.mark.gpu

M10 = 10_000_000


@pytest.fixture(scope="module")
def R10m():
    """configs[3]'s R: 10M features -> 1024, 0.32 entries per feature (73% of the rows empty)."""
    return sm.projection_operand(sm.sparse_random_matrix(1024, M10, random_state=123))


def _check(P, A, R):
    want = oracle_product(A, R)
    assert_same_csr(P.matmul(A), *want)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)


def _empty_features(R):
    return np.flatnonzero(np.diff(R.indptr) == 0)


@pytest.mark.parametrize("powerlaw", [False, True])
def test_filter_vs_oracle(R10m, powerlaw):
    rng = np.random.default_rng(300 + powerlaw)
    A = kdd_like(rng, 8000, M10, mean=99, powerlaw=powerlaw, values="normal")
    P = Projector(R10m)
    assert P.plan(A.shape[0], A.nnz)["pipeline"] == "tile"  # opt-in
    _check(P, A, R10m)
    P.set_option("filter", 1)
    assert P.plan(A.shape[0], A.nnz)["pipeline"] == "tile_filtered"
    _check(P, A, R10m)
    P.close()


def test_filter_f64_empty_rows_and_long_rows(R10m):
    """f64; empty rows; rows of only empty-R features (no product at all); rows of 3000-7000
    entries (filter units of several rounds, tiles past the caps)."""
    rng = np.random.default_rng(303)
    R = sm.projection_operand(sm.sparse_random_matrix(1024, M10, random_state=123), dtype=np.float64)
    empty = _empty_features(R)
    dead = sp.csr_matrix((rng.standard_normal(40 * 30), np.sort(rng.choice(empty, size=(40, 30)), axis=1).ravel(),
                          np.arange(0, 40 * 30 + 1, 30)), shape=(40, M10))
    A = sp.vstack([kdd_like(rng, 1500, M10, mean=99, values="normal", dtype=np.float64),
                   sp.csr_matrix((33, M10), dtype=np.float64),
                   dead,
                   kdd_like(rng, 4, M10, mean=5000, values="normal", dtype=np.float64),
                   kdd_like(rng, 900, M10, mean=99, powerlaw=True, values="normal", dtype=np.float64),
                   sp.csr_matrix((5, M10), dtype=np.float64)]).tocsr()
    P = Projector(R)
    P.set_option("filter", 1)
    _check(P, A, R)
    P.close()


@pytest.mark.parametrize("chunk_rows", [997, 2])
def test_filter_row_chunks_and_fallback(R10m, chunk_rows):
    """chunk_rows 997: ~9 row chunks, each chunk's tile 0 starting at the running total (int64
    output indptr too); 2 (below n_rows / 4096 per probe interval): the call runs unfiltered."""
    rng = np.random.default_rng(305)
    A = sp.vstack([kdd_like(rng, 4000, M10, mean=99, values="normal"),
                   sp.csr_matrix((300, M10), dtype=np.float32),
                   kdd_like(rng, 4500, M10, mean=99, powerlaw=True, values="normal")]).tocsr()
    P = Projector(R10m)
    P.set_option("filter", 1)
    P.set_option("chunk_rows", chunk_rows)
    _check(P, A, R10m)
    P.close()


def test_filter_device_int64_chunks(R10m):
    """Device path with int64 input and output indptr over several chunks, against the oracle."""
    import torch

    rng = np.random.default_rng(307)
    A = kdd_like(rng, 6000, M10, mean=99, values="normal")
    want = oracle_product(A, R10m)
    P = Projector(R10m)
    P.set_option("filter", 1)
    P.set_option("chunk_rows", 1500)
    dev = torch.device("cuda:0")
    Ap = torch.as_tensor(A.indptr.astype(np.int64), device=dev)
    Aj = torch.as_tensor(A.indices.astype(np.int32), device=dev)
    Ax = torch.as_tensor(A.data, device=dev)
    cap = int(want[1].size) + 1024
    Cp = torch.empty(A.shape[0] + 1, dtype=torch.int64, device=dev)
    Cj = torch.empty(cap, dtype=torch.int32, device=dev)
    Cx = torch.empty(cap, dtype=torch.float32, device=dev)
    nnz = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx)
    assert nnz == want[1].size
    assert np.array_equal(Cp.cpu().numpy(), want[0])
    assert np.array_equal(Cj[:nnz].cpu().numpy(), want[1])
    assert np.array_equal(Cx[:nnz].cpu().numpy().view(np.uint32), want[2].view(np.uint32))
    P.close()


@pytest.mark.parametrize("polls", [0, -1])
def test_filter_deferral(R10m, polls):
    rng = np.random.default_rng(309)
    A = kdd_like(rng, 12_000, M10, mean=99, powerlaw=True, values="normal")
    P = Projector(R10m)
    P.set_option("filter", 1)
    P.set_option("defer_polls", polls)
    _check(P, A, R10m)
    P.close()
