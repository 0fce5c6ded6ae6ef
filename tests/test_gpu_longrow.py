"""Long rows (configs[3] shape: ~100 entries, 30+ products per row; few rows per tile) against the
oracle, bit for bit — both orders, f32/f64, uniform and power-law columns, empty rows, rows beyond
the tile caps (exact slow path), frequent column collisions, forced and forbidden deferral."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import smmp
from randomprojection_amd import Projector, srp_matrix as sm
from test_gpu_parity import assert_same_csr, kdd_like, oracle_product

pytestmark = pytest.mark.gpu


def _check(P, A, R):
    want = oracle_product(A, R)
    assert_same_csr(P.matmul(A), *want)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)


@pytest.mark.parametrize("p", [1024, 4096])
@pytest.mark.parametrize("powerlaw", [False, True])
def test_longrow_vs_oracle(p, powerlaw):
    rng = np.random.default_rng(40 + p + powerlaw)
    m = 2_000_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = kdd_like(rng, 6000, m, mean=99, powerlaw=powerlaw, values="normal")
    _check(Projector(R), A, R)


def test_longrow_f64_empty_and_heavy_rows():
    rng = np.random.default_rng(77)
    m, p = 2_000_000, 4096
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123), dtype=np.float64)
    A = sp.vstack([kdd_like(rng, 700, m, mean=80, values="normal", dtype=np.float64),
                   sp.csr_matrix((40, m), dtype=np.float64),
                   kdd_like(rng, 3, m, mean=900, values="normal", dtype=np.float64),  # heavy tiles
                   kdd_like(rng, 500, m, mean=60, values="normal", dtype=np.float64)]).tocsr()
    _check(Projector(R), A, R)


def test_longrow_small_p_collisions():
    """p = 64: a row's ~40 products collide often (sums of several products, cancellation to 0)."""
    rng = np.random.default_rng(5)
    m, p = 5000, 64
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = kdd_like(rng, 3000, m, mean=60, values="normal")
    A.data[::7] = np.float32(1.0)
    _check(Projector(R), A, R)


@pytest.mark.parametrize("polls", ["0", "-1"])
def test_longrow_deferral(polls):
    rng = np.random.default_rng(9)
    m, p = 2_000_000, 1024
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = kdd_like(rng, 20_000, m, mean=99, powerlaw=True, values="normal")
    P = Projector(R)
    P.set_option("defer_polls", int(polls))
    _check(P, A, R)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_longrow_bitmap_gated_gathers(dtype):
    """The tile kernel fetches W words only for features whose R row is nonempty (feature bitmap;
    skipped entries read an out-of-range buffer offset): m not a multiple of 32, the last features
    nonempty, 70% empty R rows, rows of more than 4 entries (O records) next to empty ones."""
    rng = np.random.default_rng(123)
    m, p = (1 << 20) + 7, 1024
    live = np.sort(np.concatenate([rng.choice(m - 8, size=int(0.3 * m), replace=False), [m - 3, m - 2, m - 1]]))
    cnt = rng.choice([1, 1, 1, 2, 2, 3, 6], size=live.size)
    rows = np.repeat(live, cnt)
    cols = np.concatenate([np.sort(rng.choice(p, size=k, replace=False)) for k in cnt])
    mag = 1.5
    vals = np.where(rng.random(rows.size) < 0.5, -mag, mag).astype(dtype)
    R = sp.csr_matrix((vals, (rows, cols)), shape=(m, p))
    A = kdd_like(rng, 4000, m, mean=99, values="normal", dtype=dtype)
    tail = sp.csr_matrix((np.ones(3, dtype), (np.zeros(3, int), [m - 3, m - 2, m - 1])), shape=(1, m))
    A = sp.vstack([A, tail, A[:100]]).tocsr()
    P = Projector(R)
    assert P.layout == "packed"
    assert P.plan(A.shape[0], A.nnz)["pipeline"] == "tile"
    _check(P, A, R)
