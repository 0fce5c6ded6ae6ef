"""Chunked host streaming (rp_project_stream, boundary 2): host CSR in -> host CSR out in chunks of
rows whose upload, projection and download overlap. Checked bit for bit against the oracle
(restatement of scipy csr_matmat; reference path code/clustermode/randomProjection.py:28-54)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import same_bits
from oracle import smmp
from randomprojection_amd import Projector, srp_matrix as sm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    m, p = 2_000_000, 4096
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    rng = np.random.default_rng(31)
    n = 1_300_000
    k = 1 + rng.poisson(10, size=n)
    k[rng.integers(0, n, 2000)] = 0                      # empty rows
    indptr = np.concatenate([[0], np.cumsum(k)]).astype(np.int64)
    idx = np.sort(rng.integers(0, m, size=int(indptr[-1])).astype(np.int32))  # any order is legal input
    val = rng.standard_normal(idx.size).astype(np.float32)
    A = sp.csr_matrix((val, idx, indptr), shape=(n, m))
    return R, Projector(R), A, smmp.matmat(A, R)


@pytest.mark.parametrize("chunk", [0, 300_000, 262_144 + 17])
@pytest.mark.parametrize("order", ["scipy", "sorted"])
def test_stream_vs_oracle(setup, chunk, order):
    R, P, A, (Cp, Cj, Cx, _, _) = setup
    if order == "sorted":
        Cj, Cx = smmp.sorted_rows(Cp, Cj, Cx)
    ip, ix, dx = P.project_stream(A.indptr, A.indices, A.data, order=order, chunk_rows=chunk)
    assert np.array_equal(ip, Cp) and np.array_equal(ix, Cj) and same_bits(dx, Cx)


def test_stream_dtypes_offset_indptr_and_reused_out(setup):
    """int32 input indptr not starting at 0, int64 outputs, float64 values, caller-provided out
    arrays (too small first: the exact retry), then reused for a second call."""
    R, P, A, _ = setup
    sub = A[100_000:700_000]
    ip32 = (sub.indptr + 5).astype(np.int32)                 # indptr[0] = 5: entries start at 5
    aj = np.concatenate([np.zeros(5, np.int32), sub.indices])
    ax = np.concatenate([np.zeros(5, np.float64), sub.data.astype(np.float64)])
    Wp, Wj, Wx, _, _ = smmp.matmat(sp.csr_matrix((sub.data.astype(np.float64), sub.indices, sub.indptr),
                                                 shape=sub.shape), R)
    small = (np.empty(sub.shape[0] + 1, np.int64), np.empty(1000, np.int64), np.empty(1000, np.float64))
    ip, ix, dx = P.project_stream(ip32, aj, ax, chunk_rows=150_000, out=small)
    assert ip.dtype == np.int64 and ix.dtype == np.int64 and dx.dtype == np.float64
    assert np.array_equal(ip, Wp) and np.array_equal(ix, Wj) and same_bits(dx, Wx)
    out = (np.empty_like(ip), np.empty(Wj.size + 10, np.int64), np.empty(Wj.size + 10, np.float64))
    for _ in range(2):
        ip2, ix2, dx2 = P.project_stream(ip32, aj, ax, chunk_rows=150_000, out=out)
        assert ip2.base is not None or ip2 is out[0]
        assert np.array_equal(ip2, Wp) and np.array_equal(ix2, Wj) and same_bits(dx2, Wx)


def test_stream_chunk_beyond_slot_capacity_recomputed():
    """One chunk whose rows all hit R's longest rows: far more products than the expected-products
    capacity of a device slot, so that chunk is recomputed alone after the pipeline drains."""
    m, p = 300_000, 2048
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    heavy = np.argsort(np.diff(R.indptr))[-8:].astype(np.int32)   # the 8 densest R rows
    rng = np.random.default_rng(5)
    n1, n2 = 400_000, 200_000
    k1 = 1 + rng.poisson(5, size=n1)
    cols1 = np.sort(rng.integers(0, m, size=int(k1.sum())).astype(np.int32))
    cols2 = np.tile(np.sort(heavy), n2)
    indptr = np.concatenate([[0], np.cumsum(k1), k1.sum() + 8 * np.arange(1, n2 + 1)]).astype(np.int64)
    A = sp.csr_matrix((rng.standard_normal(indptr[-1]).astype(np.float32), np.concatenate([cols1, cols2]), indptr),
                      shape=(n1 + n2, m))
    Cp, Cj, Cx, _, _ = smmp.matmat(A, R)
    ip, ix, dx = P.project_stream(A.indptr, A.indices, A.data, chunk_rows=100_000)
    assert np.array_equal(ip, Cp) and np.array_equal(ix, Cj) and same_bits(dx, Cx)
    # chunks 4 and 5 are the heavy ones; when they launch only uniform chunks have come back
    assert P.stream_stats() == {"chunks": 6, "recomputed": 2, "regrown": 0}


def test_stream_slots_follow_measured_output():
    """Every row hits R's densest rows (~3x the outputs per entry R's mean row length predicts):
    the first kStreamSlots = 3 chunks are launched before any has come back and are recomputed;
    from then on each slot grows to the measured output per entry before it takes its next chunk,
    so no later chunk is recomputed. Bit-exact either way (scipy csr_matmat, the oracle)."""
    m, p = 300_000, 2048
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    heavy = np.argsort(np.diff(R.indptr))[-64:].astype(np.int32)
    rng = np.random.default_rng(7)
    n = 500_000
    k = 1 + rng.poisson(6, size=n)
    cols = [np.unique(rng.choice(heavy, size=int(x))) for x in k]
    indptr = np.concatenate([[0], np.cumsum([c.size for c in cols])]).astype(np.int64)
    A = sp.csr_matrix((rng.standard_normal(indptr[-1]).astype(np.float32), np.concatenate(cols), indptr),
                      shape=(n, m))
    Cp, Cj, Cx, _, _ = smmp.matmat(A, R)
    ip, ix, dx = P.project_stream(A.indptr, A.indices, A.data, chunk_rows=50_000)
    assert np.array_equal(ip, Cp) and np.array_equal(ix, Cj) and same_bits(dx, Cx)
    st = P.stream_stats()
    assert st["chunks"] == 10 and st["recomputed"] == 3 and 3 <= st["regrown"] <= 7, st


def test_stream_errors(setup):
    R, P, A, _ = setup
    bad = A.indices.copy()
    bad[-3] = P.m + 7                                      # in the last chunk
    with pytest.raises(ValueError, match="out of range"):
        P.project_stream(A.indptr, bad, A.data, chunk_rows=200_000)
    ip = A.indptr.copy()
    ip[500_001] = ip[500_000] - 1                           # decreasing inside a chunk
    with pytest.raises(ValueError, match="decreasing"):
        P.project_stream(ip, A.indices, A.data, chunk_rows=200_000)
    # still usable afterwards
    C = P.project_stream(A.indptr[:1001], A.indices, A.data)
    assert C[0].size == 1001


def test_matmul_routes_large_inputs_through_stream(setup, monkeypatch):
    import randomprojection_amd.projector as pj

    R, P, A, (Cp, Cj, Cx, _, _) = setup
    monkeypatch.setattr(pj, "STREAM_MIN_ROWS", 1000)
    C = P.matmul(A)
    assert isinstance(C, sp.csr_matrix)
    assert np.array_equal(C.indptr, Cp) and np.array_equal(C.indices, Cj) and same_bits(C.data, Cx)
