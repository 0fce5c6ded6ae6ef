"""Staged gather: bucketed descriptor fetch for the row-lane pipeline (super-tile
partition with per-unit run parts, bitmap-filtered gather, wave kernel reading its unit's parts of
the runs), and the tile
pipeline under the same staging requests (it gathers directly since round 4: a staging request is
accepted and ignored there). Results must be bit-identical to the direct-gather kernels and to the
oracle (CPU restatement of scipy csr_matmat) for every bucket width, order, dtype, tile shape and
workspace arrangement."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import smmp
from randomprojection_amd import Projector, srp_matrix as sm
from test_gpu_parity import assert_same_csr, kdd_like, oracle_product

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R2m():
    return sm.projection_operand(sm.sparse_random_matrix(4096, 2_000_000, random_state=123))


@pytest.fixture(scope="module")
def R2m_p1k():
    """2M features -> 1024: 0.72 R entries per feature, so KDD-like rows (11 entries, 8 products)
    qualify for the row-lane pipeline (<= 24 products per row); R2m's 2.9 per feature do not."""
    return sm.projection_operand(sm.sparse_random_matrix(1024, 2_000_000, random_state=123))


def _staged(R, shift, **kw):
    P = Projector(R, **kw)
    P.set_staging("on", shift)
    return P


@pytest.mark.parametrize("shift", [13, 16, 19])
@pytest.mark.parametrize("powerlaw", [False, True])
def test_staged_kdd_vs_oracle(R2m, shift, powerlaw):
    rng = np.random.default_rng(100 + shift + powerlaw)
    A = kdd_like(rng, 60_000, R2m.shape[0], powerlaw=powerlaw, values="normal")
    P = _staged(R2m, shift)
    assert P.plan(A.shape[0], A.nnz) == {"pipeline": "tile", "staged": False, "bucket_shift": 0}
    want = oracle_product(A, R2m)
    assert_same_csr(P.matmul(A), *want)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)


def test_staged_f64_and_heavy_tiles():
    """f64 compute, rows past the LDS caps (exact slow path, no staged runs) mixed with short rows."""
    rng = np.random.default_rng(21)
    m, p = 5000, 64
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123), dtype=np.float64)
    parts = [kdd_like(rng, 300, m, mean=10, values="normal", dtype=np.float64),
             kdd_like(rng, 3, m, mean=900, values="normal", dtype=np.float64, cap=m),
             kdd_like(rng, 20, m, mean=300, values="normal", dtype=np.float64),
             sp.csr_matrix((50, m), dtype=np.float64),
             kdd_like(rng, 400, m, mean=3, values="normal", dtype=np.float64)]
    A = sp.vstack(parts).tocsr()
    for shift in (5, 8, 12):
        P = _staged(R, shift)
        for order in ("scipy", "sorted"):
            Cp, Cj, Cx = oracle_product(A, R)
            if order == "sorted":
                Cj, Cx = smmp.sorted_rows(Cp, Cj, Cx)
            assert_same_csr(P.matmul(A, order=order), Cp, Cj, Cx)


def test_staged_equals_direct_cfg4_shape():
    """100 nnz/row power-law rows over p=1024 (config 4 shape, m scaled to 2M): the tile pipeline with
    and without a staging request gives the same bits."""
    rng = np.random.default_rng(4)
    m, p = 2_000_000, 1024
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = kdd_like(rng, 4000, m, mean=99, powerlaw=True, values="normal")
    direct = Projector(R)
    direct.set_staging("off")
    Cd = direct.matmul(A)
    Cs = _staged(R, 15).matmul(A)
    assert_same_csr(Cs, Cd.indptr, Cd.indices, Cd.data)
    assert_same_csr(Cs, *oracle_product(A, R))


def test_staged_device_path_workspace_and_offset_indptr(R2m):
    """Caller workspace: large enough -> staged; too small for staging -> direct; indptr[0] != 0."""
    import torch

    rng = np.random.default_rng(8)
    A = kdd_like(rng, 30_000, R2m.shape[0], values="normal")
    P = _staged(R2m, 17)
    dev = torch.device("cuda", 0)
    want = oracle_product(A, R2m)
    skip = 1000  # rows [skip:] through an indptr whose first value is A.indptr[skip] (not 0)
    sub = A[skip:]
    want_sub = oracle_product(sub, R2m)
    for small in (False, True):
        for base in (0, skip):
            Ap = torch.as_tensor(A.indptr[base:].astype(np.int64), device=dev)
            Aj = torch.as_tensor(A.indices, device=dev)
            Ax = torch.as_tensor(A.data, device=dev)
            n = A.shape[0] - base
            nnz = int(A.indptr[-1] - A.indptr[base])
            full = P.workspace_bytes(n, nnz)
            ws = torch.empty(P.workspace_bytes(n) if small else full, dtype=torch.uint8, device=dev)
            cap = 4 * nnz  # >= output nnz for this R (2.9 products per entry)
            Cp = torch.empty(n + 1, dtype=torch.int64, device=dev)
            Cj = torch.empty(cap, dtype=torch.int32, device=dev)
            Cx = torch.empty(cap, dtype=torch.float32, device=dev)
            k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, workspace=ws, nnz_a=nnz)
            torch.cuda.synchronize()
            ref = want if base == 0 else want_sub
            got = sp.csr_matrix((Cx[:k].cpu().numpy(), Cj[:k].cpu().numpy(), Cp.cpu().numpy()),
                                shape=(n, R2m.shape[1]))
            assert_same_csr(got, *ref)


def test_staging_arguments():
    from randomprojection_amd import _native as nat

    R = sm.projection_operand(sm.sparse_random_matrix(64, 100_000, random_state=123))
    P = Projector(R)
    with pytest.raises(nat.RPError):
        P.set_staging("on", 8)       # 391 buckets > 256
    with pytest.raises(nat.RPError):
        P.set_staging("on", 21)
    G = Projector(R, layout="generic")
    with pytest.raises(nat.RPError):
        G.set_staging("on")
    G.set_staging("off")
    P.set_staging("auto")


@pytest.mark.parametrize("polls", ["0", "-1", "3"])
@pytest.mark.parametrize("staged", [False, True])
def test_deferred_output_tiles(R2m, polls, staged):
    """Tiles that park their output (option defer_polls=0: nearly all) and tiles that wait (-1)
    give the same bits; mixed with heavy tiles, empty rows, both orders."""
    rng = np.random.default_rng(31)
    m = R2m.shape[0]
    A = sp.vstack([kdd_like(rng, 20_000, m, values="normal"), sp.csr_matrix((300, m), dtype=np.float32),
                   kdd_like(rng, 40, m, mean=300, values="normal"),
                   kdd_like(rng, 20_000, m, powerlaw=True, values="normal")]).tocsr()
    P = _staged(R2m, 16) if staged else Projector(R2m)
    P.set_option("defer_polls", int(polls))
    want = oracle_product(A, R2m)
    assert_same_csr(P.matmul(A), *want)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)


@pytest.mark.parametrize("ticks", ["1", "300", "100000"])
def test_deferred_output_time_budget(R2m, ticks):
    """256-row tiles wait up to defer_ticks s_memrealtime ticks (default 800 = 8 us) before
    parking their output: every budget gives the oracle's bits."""
    rng = np.random.default_rng(57)
    m = R2m.shape[0]
    A = sp.vstack([kdd_like(rng, 25_000, m, values="normal"), sp.csr_matrix((200, m), dtype=np.float32),
                   kdd_like(rng, 25_000, m, powerlaw=True, values="normal")]).tocsr()
    want = oracle_product(A, R2m)
    P = Projector(R2m)
    P.set_option("defer_ticks", int(ticks))
    assert_same_csr(P.matmul(A), *want)


@pytest.mark.parametrize("pipe", ["tile", "lpr"])
def test_pipelines_multi_group_vs_oracle(R2m_p1k, pipe):
    """Each pipeline forced (option pipeline), direct and staged, over 600k rows: 2344 row-lane tiles, so
    the staged gather spans three 1024-tile groups and ends in a partial one; uniform and
    power-law rows, empty rows, both orders."""
    rng = np.random.default_rng(77)
    R = R2m_p1k
    m = R.shape[0]
    A = sp.vstack([kdd_like(rng, 300_000, m, values="normal"), sp.csr_matrix((777, m), dtype=np.float32),
                   kdd_like(rng, 299_223, m, powerlaw=True, values="normal")]).tocsr()
    want = oracle_product(A, R)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    for stage in ("off", "on"):
        P = Projector(R)
        P.set_option("pipeline", "rowlane" if pipe == "lpr" else "tile")
        P.set_staging(stage, 19)
        assert P.plan(A.shape[0], A.nnz)["pipeline"] == ("rowlane" if pipe == "lpr" else "tile")
        assert_same_csr(P.matmul(A), *want)
        assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)
        P.close()


@pytest.mark.parametrize("chunk", ["256", "50000"])
def test_rowlane_chunked_launch_vs_oracle(R2m_p1k, chunk):
    """The row-lane pipeline over several row chunks (option chunk_rows; huge launches such as
    configs[2]'s 1.08B rows run in chunks of 2^27): every chunk writes its indptr slice and its
    entries at the running total of the chunks before it. Ragged last chunk, empty rows at a chunk
    boundary, heavy rows, direct and staged, both orders, int64 output indptr."""
    rng = np.random.default_rng(91)
    R = R2m_p1k
    m = R.shape[0]
    n1 = 50_176 if chunk == "50000" else 1024
    A = sp.vstack([kdd_like(rng, n1 - 300, m, values="normal"), sp.csr_matrix((600, m), dtype=np.float32),
                   kdd_like(rng, 2, m, mean=3000, values="normal", cap=m),
                   kdd_like(rng, 123_321 if chunk == "50000" else 3001, m, powerlaw=True, values="normal")]).tocsr()
    want = oracle_product(A, R)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    for stage in ("off", "on"):
        P = Projector(R)
        P.set_option("pipeline", "rowlane")
        P.set_option("chunk_rows", int(chunk))
        P.set_staging(stage, 19)
        assert P.plan(A.shape[0], A.nnz) == {"pipeline": "rowlane", "staged": stage == "on",
                                             "bucket_shift": 19 if stage == "on" else 0}
        assert_same_csr(P.matmul(A), *want)
        assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)
        P.close()
    _device_int64_indptr_vs_oracle(R, A, want)


def _device_int64_indptr_vs_oracle(R, A, want):
    import torch

    P = Projector(R)
    dev = torch.device("cuda", 0)
    Ap = torch.as_tensor(A.indptr.astype(np.int64), device=dev)
    Aj = torch.as_tensor(A.indices.astype(np.int32), device=dev)
    Ax = torch.as_tensor(A.data, device=dev)
    n, cap = A.shape[0], int(want[0][-1]) + 100
    Cp = torch.empty(n + 1, dtype=torch.int64, device=dev)
    Cj = torch.empty(cap, dtype=torch.int64, device=dev)
    Cx = torch.empty(cap, dtype=torch.float32, device=dev)
    ws = torch.empty(P.workspace_bytes(n, A.nnz), dtype=torch.uint8, device=dev)
    nnz = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, workspace=ws, nnz_a=A.nnz)
    assert nnz == int(want[0][-1])
    assert np.array_equal(Cp.cpu().numpy(), want[0].astype(np.int64))
    assert np.array_equal(Cj[:nnz].cpu().numpy(), want[1].astype(np.int64))
    assert np.array_equal(Cx[:nnz].cpu().numpy().view(np.uint32), want[2].view(np.uint32))
    P.close()


def test_rowlane_staged_tile_past_one_round(R2m_p1k):
    """A tile of 3088 entries (> 12 x 256 = one round of the staged descriptor fetch, <= the entry
    cap): the second round runs with 16 of 256 lanes in range. Regression: the run lookup shuffled
    from lanes that had left the loop (found on 500M-row runs: one tile in ~1M)."""
    rng = np.random.default_rng(3088)
    R = R2m_p1k
    m = R.shape[0]
    k = np.full(256, 12)
    k[:16] = 13
    cols = [np.sort(rng.choice(m, size=int(x), replace=False)) for x in k]
    heavy = sp.csr_matrix((rng.standard_normal(int(k.sum())).astype(np.float32), np.concatenate(cols),
                           np.concatenate([[0], np.cumsum(k)])), shape=(256, m))
    A = sp.vstack([kdd_like(rng, 17 * 256, m, values="normal"), heavy,
                   kdd_like(rng, 22 * 256 + 77, m, values="normal")]).tocsr()
    want = oracle_product(A, R)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    P = Projector(R)
    P.set_option("pipeline", "rowlane")
    P.set_staging("on", 16)
    assert P.plan(A.shape[0], A.nnz)["staged"]
    assert_same_csr(P.matmul(A), *want)
    assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)
    P.close()


def _rows(rng, k, pool, m, dtype=np.float32):
    """CSR rows with k[i] distinct columns drawn from `pool` (ascending), normal values."""
    k = np.asarray(k)
    n, kmax, big = len(k), int(k.max()), np.iinfo(np.int64).max
    valid = np.arange(kmax)[None, :] < k[:, None]
    draw = np.full((n, kmax), big)
    todo = np.arange(n)
    while todo.size:  # redraw the rows that drew a column twice
        d = np.where(valid[todo], rng.integers(0, len(pool), size=(todo.size, kmax)), big)
        d.sort(axis=1)
        draw[todo] = d
        todo = todo[((np.diff(d, axis=1) == 0) & valid[todo][:, 1:]).any(axis=1)]
    cols = np.asarray(pool, dtype=np.int64)[draw[valid]]
    return sp.csr_matrix((rng.standard_normal(int(k.sum())).astype(dtype), cols,
                          np.concatenate([[0], np.cumsum(k)])), shape=(n, m))


def _check_rowlane_staged(R, A, shift, staged=True):
    """Row-lane pipeline with staging forced on: host path in both orders against the oracle, then
    the device path, whose workspace records whether the staged gather ran (`staged`) or a segment
    past its reserve sent the call to direct gathers."""
    import torch

    want = oracle_product(A, R)
    Cj, Cx = smmp.sorted_rows(want[0], want[1], want[2])
    P = Projector(R)
    P.set_option("pipeline", "rowlane")
    P.set_staging("on", shift)
    assert P.plan(A.shape[0], A.nnz) == {"pipeline": "rowlane", "staged": True, "bucket_shift": shift}
    assert_same_csr(P.matmul(A), *want)
    assert_same_csr(P.matmul(A, order="sorted"), want[0], Cj, Cx)
    dev = torch.device("cuda", 0)
    n, nnz = A.shape[0], int(want[0][-1])
    Ap = torch.as_tensor(A.indptr.astype(np.int32), device=dev)
    Aj = torch.as_tensor(A.indices.astype(np.int32), device=dev)
    Ax = torch.as_tensor(A.data, device=dev)
    ws = torch.empty(P.workspace_bytes(n, A.nnz), dtype=torch.uint8, device=dev)
    Cp_d = torch.empty(n + 1, dtype=torch.int32, device=dev)
    Cj_d = torch.empty(nnz + 64, dtype=torch.int32, device=dev)
    Cx_d = torch.empty(nnz + 64, dtype=torch.float32, device=dev)
    assert P.project_device(Ap, Aj, Ax, Cp_d, Cj_d, Cx_d, workspace=ws, nnz_a=A.nnz) == nnz
    assert P.choice(n, A.nnz, ws) == staged
    got = sp.csr_matrix((Cx_d[:nnz].cpu().numpy(), Cj_d[:nnz].cpu().numpy(), Cp_d.cpu().numpy()), shape=(n, R.shape[1]))
    assert_same_csr(got, *want)
    P.close()


def test_rowlane_staged_tile_of_3200_live_entries(R2m_p1k):
    """A tile of 3200 entries, all on nonempty R rows (every staged word carries products): its
    words take two rounds of the main kernel's descriptor fetch (12 x 256 per round), the second
    with 128 of 256 lanes in range, next to tiles of ~11 entries per row."""
    rng = np.random.default_rng(3200)
    R = R2m_p1k
    m = R.shape[0]
    live = np.flatnonzero(np.diff(R.indptr) > 0)
    k = np.full(256, 12)
    k[:128] = 13
    A = sp.vstack([kdd_like(rng, 9 * 256, m, mean=11.2, values="normal"), _rows(rng, k, live, m),
                   kdd_like(rng, 9 * 256 + 31, m, mean=11.2, values="normal")]).tocsr()
    _check_rowlane_staged(R, A, 16)


def test_rowlane_staged_wave_edges(R2m_p1k):
    """The staged wave kernel on edge cases: a 64-row unit of 2240 entries (past the unit cap: the
    tile goes to the exact heavy path) next to light units of its tile, a unit whose 64 rows each
    hold one feature with more than 2 R entries plus ordinary ones (more side entries than the
    wave's side list: heavy), units of 13 steps, empty rows, both orders."""
    rng = np.random.default_rng(5)
    R = R2m_p1k
    m = R.shape[0]
    rl = np.diff(R.indptr)
    side, live = np.flatnonzero(rl >= 3), np.flatnonzero(rl > 0)
    big = sp.vstack([_rows(rng, np.full(64, 35), np.arange(m), m), _rows(rng, np.full(192, 3), np.arange(m), m)])
    top = (_rows(rng, np.ones(64, int), side, m) + _rows(rng, np.full(64, 4), live, m)).tocsr()
    top.sort_indices()
    sidey = sp.vstack([top, _rows(rng, np.full(192, 9), np.arange(m), m)])
    A = sp.vstack([kdd_like(rng, 5 * 256, m, values="normal"), big, _rows(rng, np.full(256, 13), np.arange(m), m),
                   sp.csr_matrix((70, m), dtype=np.float32), sidey.astype(np.float32),
                   kdd_like(rng, 7 * 256 + 9, m, values="normal")]).tocsr()
    _check_rowlane_staged(R, A, 16)
    _check_rowlane_staged(R, sp.vstack([kdd_like(rng, 9 * 256 + 5, m, mean=11.2, values="normal")]).tocsr(), 19)


def test_rowlane_staged_zero_values_and_empty_rows(R2m_p1k):
    """Explicit zeros (+0.0 and -0.0, ~4% of the values, some rows all zero) among KDD-like rows
    with empty rows between them: a zero value's products are not in the slot, so its row is
    rebuilt by the wave kernel's exact path (rows flagged by their ordinal among the unit's
    nonempty rows, mapped back to row lanes after the flat pass)."""
    rng = np.random.default_rng(4040)
    R = R2m_p1k
    m = R.shape[0]
    A = kdd_like(rng, 12 * 256 + 17, m, mean=11.2, values="normal").tolil()
    A[rng.choice(A.shape[0], 400, replace=False)] = 0  # empty rows between nonempty ones
    A = A.tocsr()
    A.sort_indices()
    z = rng.random(A.nnz) < 0.04
    A.data[z] = np.where(rng.random(int(z.sum())) < 0.5, 0.0, -0.0).astype(np.float32)
    for r in rng.choice(A.shape[0], 40, replace=False):  # rows of zeros only
        A.data[A.indptr[r]:A.indptr[r + 1]] = 0.0
    assert A.nnz == int(A.indptr[-1])  # the explicit zeros stay stored
    _check_rowlane_staged(R, A, 16)


@pytest.mark.parametrize("k", [15, 16, 17])
def test_rowlane_staged_unit_cap(R2m_p1k, k):
    """Units at the wave kernel's register cap: 64 rows of k entries (k = 16: exactly 16 steps of 64
    = the cap, the fast path; 17: one step past it, the tile goes heavy; 15: one step below), with
    side entries and repeated output columns, next to ordinary tiles; a run table with entries of
    all four units in most buckets."""
    rng = np.random.default_rng(1600 + k)
    R = R2m_p1k
    m = R.shape[0]
    rl = np.diff(R.indptr)
    side = np.flatnonzero(rl >= 3)
    wide = (_rows(rng, np.full(64, k - 1), np.arange(m), m) + _rows(rng, np.ones(64, int), side, m)).tocsr()
    wide.sort_indices()
    A = sp.vstack([kdd_like(rng, 3 * 256 + 64, m, mean=11.2, values="normal"), wide.astype(np.float32),
                   kdd_like(rng, 128 + 5 * 256, m, mean=11.2, values="normal")]).tocsr()
    _check_rowlane_staged(R, A, 17)


def test_rowlane_staged_dead_tiles_and_empty_rows(R2m_p1k):
    """Tiles none of whose entries has a nonempty R row (every staged word filtered by the gather's
    bitmap, no products) among ~1500 tiles of uniform columns over 245 buckets, plus empty rows: the
    segment reserves hold (binomial counts), the staged gather runs."""
    rng = np.random.default_rng(1500)
    R = R2m_p1k
    m = R.shape[0]
    dead = np.flatnonzero(np.diff(R.indptr) == 0)
    A = sp.vstack([_rows(rng, np.full(256 * 600, 3), np.arange(m), m), _rows(rng, np.full(3 * 256, 4), dead, m),
                   sp.csr_matrix((300, m), dtype=np.float32), _rows(rng, np.full(256 * 900, 3), np.arange(m), m)]).tocsr()
    _check_rowlane_staged(R, A, 13)


def test_rowlane_staged_segment_overflow_goes_direct(R2m_p1k):
    """Staging forced on columns far from uniform (every entry in the first two of 245 buckets):
    the first tiles' runs exceed their segments' reserves, the partition clears the gate and the
    direct kernel projects the call; the output is the oracle's either way."""
    rng = np.random.default_rng(245)
    R = R2m_p1k
    m = R.shape[0]
    A = _rows(rng, np.full(256 * 300, 5), np.arange(2 << 13), m)
    _check_rowlane_staged(R, A, 13, staged=False)


@pytest.mark.parametrize("dist", ["uniform", "powerlaw"])
def test_auto_staging_choice_on_device(dist):
    """Auto mode on a launch large enough to stage (>= 4M entries, R's W table >= 64 MB): the device
    samples the feature ids and picks the staged gather for uniform columns, direct gathers for
    power-law ones; staging forced on power-law columns overflows the hot features' segment
    reserves and goes direct too. Either way the whole output equals the oracle's."""
    import torch
    from randomprojection_amd import synth

    m, p, n = 10_000_000, 256, 420_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    Ap, Aj, Ax = synth.kdd_rows_device(n, m, seed=33, dist=dist)
    nnz_a = int(Aj.numel())
    outs = {}
    for mode in ("auto", "on", "off"):
        P = Projector(R)
        P.set_staging(mode)
        plan = P.plan(n, nnz_a)
        assert plan["pipeline"] == "rowlane" and plan["staged"] == {"auto": "auto", "on": True, "off": False}[mode]
        ws = torch.empty(P.workspace_bytes(n, nnz_a), dtype=torch.uint8, device="cuda")
        cap = int(3 * nnz_a * P.nnz / P.m) + 65536  # hot power-law features may carry more R entries
        Cp = torch.empty(n + 1, dtype=torch.int32, device="cuda")
        Cj = torch.empty(cap, dtype=torch.int32, device="cuda")
        Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
        k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, workspace=ws, nnz_a=nnz_a)
        # what ran is recorded in the workspace by every call, forced modes included
        assert P.choice(n, nnz_a, ws) == {"auto": dist == "uniform", "on": dist == "uniform", "off": False}[mode]
        outs[mode] = (Cp.cpu().numpy(), Cj[:k].cpu().numpy(), Cx[:k].cpu().numpy())
        P.close()
    A = sp.csr_matrix((Ax.cpu().numpy(), Aj.cpu().numpy(), Ap.cpu().numpy()), shape=(n, m))
    want = oracle_product(A, R)
    for mode, (cp, cj, cx) in outs.items():
        assert np.array_equal(cp, want[0]) and np.array_equal(cj, want[1]), mode
        assert np.array_equal(cx.view(np.uint32), want[2].view(np.uint32)), mode


@pytest.mark.parametrize("dist", ["uniform", "powerlaw"])
def test_auto_staging_async_and_graph_capture(dist):
    """Auto mode without total_nnz (``sync=False``) never waits on the host: the sampled verdict stays
    on the device and gates the staged kernels (power-law columns: the reserve/partition/gather
    kernels return at once and the wave kernel gathers directly). The same call captured in a HIP
    graph and replayed gives the same bits; the sync form's output is the reference (the oracle
    checks it in test_auto_staging_choice_on_device). Under capture, a call that would wait on the
    host (total_nnz asked) is refused before anything is enqueued."""
    import torch
    from randomprojection_amd import _native as nat
    from randomprojection_amd import synth

    m, p, n = 10_000_000, 256, 420_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    Ap, Aj, Ax = synth.kdd_rows_device(n, m, seed=34, dist=dist)
    nnz_a = int(Aj.numel())
    P = Projector(R)
    assert P.plan(n, nnz_a)["staged"] == "auto"
    ws = torch.empty(P.workspace_bytes(n, nnz_a), dtype=torch.uint8, device="cuda")
    cap = int(3 * nnz_a * P.nnz / P.m) + 65536

    def outs():
        return (torch.empty(n + 1, dtype=torch.int32, device="cuda"), torch.empty(cap, dtype=torch.int32, device="cuda"),
                torch.empty(cap, dtype=torch.float32, device="cuda"))

    Cp, Cj, Cx = outs()
    k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, workspace=ws, nnz_a=nnz_a)
    ref = (Cp.clone(), Cj[:k].clone(), Cx[:k].clone())
    side = torch.cuda.Stream()
    Dp, Dj, Dx = outs()
    with torch.cuda.stream(side):
        assert P.project_device(Ap, Aj, Ax, Dp, Dj, Dx, workspace=ws, nnz_a=nnz_a, stream=side.cuda_stream,
                                sync=False) is None
    side.synchronize()
    assert P.choice(n, nnz_a, ws) == (dist == "uniform")
    assert torch.equal(Dp, ref[0]) and torch.equal(Dj[:k], ref[1]) and torch.equal(Dx[:k].view(torch.int32),
                                                                                 ref[2].view(torch.int32))
    Gp, Gj, Gx = outs()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        P.project_device(Ap, Aj, Ax, Gp, Gj, Gx, workspace=ws, nnz_a=nnz_a, stream=side.cuda_stream, sync=False)
        with pytest.raises(nat.RPError, match="stream capture"):
            P.project_device(Ap, Aj, Ax, Gp, Gj, Gx, workspace=ws, nnz_a=nnz_a, stream=side.cuda_stream)
    for _ in range(2):
        Gj.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(Gp, ref[0]) and torch.equal(Gj[:k], ref[1]) and torch.equal(Gx[:k].view(torch.int32),
                                                                                     ref[2].view(torch.int32))
    del g
    P.close()
