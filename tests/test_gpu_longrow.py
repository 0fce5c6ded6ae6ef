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
@pytest.mark.parametrize("p", [64, 1024, 2048])
def test_longrow_wave_pipeline_vs_oracle(dtype, p):
    """The long-row wave pipeline (one wave per tile of rows, LDS first-touch table) forced and
    chosen automatically, against the oracle and against the tile pipeline on the same rows: long
    rows, empty rows, rows past the wave's caps (more than 256 entries or 256 products: the tile
    goes to the heavy kernel), short rows between them, int32 and int64 output indptr."""
    rng = np.random.default_rng(123 + p)
    m = 4_000_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=7), dtype=dtype)
    ppe = R.nnz / m
    heavy = kdd_like(rng, 3, m, mean=min(m - 1, int(300 / max(ppe, 0.05))), values="normal", dtype=dtype,
                     cap=m)  # > 256 products
    A = sp.vstack([kdd_like(rng, 4000, m, mean=99, values="normal", dtype=dtype),
                   sp.csr_matrix((37, m), dtype=dtype),
                   heavy,
                   kdd_like(rng, 2, m, mean=600, values="normal", dtype=dtype, cap=m),  # > 256 entries
                   kdd_like(rng, 500, m, mean=3, values="normal", dtype=dtype),
                   kdd_like(rng, 3000, m, mean=120, powerlaw=True, values="normal", dtype=dtype)]).tocsr()
    want = oracle_product(A, R)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    P = Projector(R)
    assert P.plan(A.shape[0], A.nnz)["pipeline"] == "longrow"
    for pipe in ("auto", "longrow", "tile"):
        P.set_option("pipeline", pipe)
        assert_same_csr(P.matmul(A), *want)
        assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)
    P.set_option("pipeline", None)


@pytest.mark.parametrize("polls", [0, 3, -1])
def test_longrow_wave_deferral_and_flags(polls):
    """Wave tiles that park their output at once (0 polls), after a few, or with the long budget
    that stands in for "never" (-1): the same bits; heavy tiles between them make successors wait
    for tiles that publish only in the heavy kernel."""
    rng = np.random.default_rng(31)
    m, p = 1_000_000, 1024
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = sp.vstack([kdd_like(rng, 5000, m, mean=99, values="normal"),
                   kdd_like(rng, 1, m, mean=1500, values="normal", cap=m),
                   kdd_like(rng, 5000, m, mean=99, powerlaw=True, values="normal"),
                   kdd_like(rng, 1, m, mean=1500, values="normal", cap=m),
                   kdd_like(rng, 700, m, mean=99, values="normal")]).tocsr()
    P = Projector(R)
    P.set_option("defer_polls", polls)
    assert P.plan(A.shape[0], A.nnz)["pipeline"] == "longrow"
    _check(P, A, R)
