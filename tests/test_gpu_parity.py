"""GPU parity: librp's HIP SpGEMM against scipy-made golden vectors, the oracle (CPU restatement of
scipy csr_matmat) and sklearn — bit for bit (structure, order and value bits)."""
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr, golden_R, same_bits
from oracle import smmp
from randomprojection_amd import Projector, srp_matrix as sm
from randomprojection_amd import random_project_map_function, random_project_mappartitions_function
from randomprojection_amd.linalg import SparseVector

warnings.filterwarnings("ignore")
pytestmark = pytest.mark.gpu

CASES = ["kdd_ones", "kdd_vals", "adv_f32", "vals_f64", "mixed_f32xf64", "adv_f64"]


def assert_same_csr(C, Cp, Cj, Cx):
    assert np.array_equal(C.indptr, Cp), "indptr"
    assert np.array_equal(C.indices, Cj), "indices"
    assert same_bits(C.data, Cx), "data bits"


def oracle_product(A, R):
    Cp, Cj, Cx, _, _ = smmp.matmat(A, R)
    return Cp, Cj, Cx


def kdd_like(rng, n, m, mean=10.0, powerlaw=False, values="ones", dtype=np.float32, cap=None):
    k = 1 + rng.poisson(mean, size=n)
    if cap:
        k = np.minimum(k, cap)
    indptr = np.zeros(n + 1, np.int64)
    indptr[1:] = np.cumsum(k)
    if powerlaw:
        # Zipf(1.1) ranks over a fixed permutation, without replacement inside a row
        perm = rng.permutation(m)
        cdf = np.cumsum(1.0 / np.arange(1, m + 1) ** 1.1)
        cdf /= cdf[-1]
        cols = []
        for x in k:
            x = int(min(x, m))
            got = np.zeros(0, np.int64)
            while got.size < x:
                draws = np.searchsorted(cdf, rng.random(2 * x + 4))
                _, first = np.unique(np.concatenate([got, draws]), return_index=True)
                got = np.concatenate([got, draws])[np.sort(first)]
            cols.append(np.sort(perm[got[:x]]))
        k = np.array([c.size for c in cols])
        indptr[1:] = np.cumsum(k)
    else:
        cols = []
        for x in k:
            c = np.unique(rng.integers(0, m, size=int(x)))
            cols.append(c)
        k = np.array([c.size for c in cols])
        indptr[1:] = np.cumsum(k)
    idx = np.concatenate(cols).astype(np.int32)
    val = np.ones(idx.size, dtype) if values == "ones" else rng.standard_normal(idx.size).astype(dtype)
    return sp.csr_matrix((val, idx, indptr), shape=(n, m))


@pytest.fixture(scope="module")
def projectors(golden):
    out = {}
    for which in (1, 2):
        R = golden_R(golden, which)
        out[(which, "auto")] = Projector(R)
        out[(which, "generic")] = Projector(R, layout="generic")
    return out


def test_layouts_selected(projectors):
    assert projectors[(1, "auto")].layout == "packed"
    assert projectors[(2, "auto")].layout == "packed"
    assert projectors[(1, "generic")].layout == "generic"


@pytest.mark.parametrize("layout", ["auto", "generic"])
@pytest.mark.parametrize("name", CASES)
def test_golden_scipy_order(golden, projectors, name, layout):
    A = golden_csr(golden, "A_" + name)
    P = projectors[(int(golden["R_" + name][0]), layout)]
    C = P.matmul(A)
    assert isinstance(C, sp.csr_matrix)
    assert C.dtype == golden["C_" + name + "_data"].dtype
    assert C.indices.dtype == golden["C_" + name + "_indices"].dtype
    assert_same_csr(C, golden["C_" + name + "_indptr"], golden["C_" + name + "_indices"],
                    golden["C_" + name + "_data"])


@pytest.mark.parametrize("layout", ["auto", "generic"])
@pytest.mark.parametrize("name", CASES)
def test_golden_sorted_order(golden, projectors, name, layout):
    A = golden_csr(golden, "A_" + name)
    P = projectors[(int(golden["R_" + name][0]), layout)]
    C = P.matmul(A, order="sorted")
    assert_same_csr(C, golden["C_" + name + "_indptr"], golden["Csorted_" + name + "_indices"],
                    golden["Csorted_" + name + "_data"])


def test_partition_function_matches_reference(golden):
    A = golden_csr(golden, "A_kdd_vals")[:300]
    R = golden_R(golden, 1)
    rows = []
    for i in range(A.shape[0]):
        s, e = A.indptr[i], A.indptr[i + 1]
        rows.append({"id": 1000 + 7 * i, "label": float(i % 2),
                     "features": SparseVector(A.shape[1], A.indices[s:e], A.data[s:e].astype(np.float64))})
    out = list(random_project_mappartitions_function(iter(rows), R))
    ptr = golden["ref_part_indptr"]
    assert len(out) == 300
    for i, (rid, lab, vec) in enumerate(out):
        assert rid == golden["ref_part_ids"][i] and lab == golden["ref_part_labels"][i]
        assert vec.size == int(golden["ref_part_size"][0])
        assert np.array_equal(vec.indices, golden["ref_part_indices"][ptr[i]:ptr[i + 1]])
        assert same_bits(vec.values, golden["ref_part_values"][ptr[i]:ptr[i + 1]])
    # the no-label branch: the reference raises TypeError; the drop-in yields (id, vector)
    nol = list(random_project_mappartitions_function(iter([{"id": 5, "features": rows[0]["features"]}]), R))
    assert nol[0][0] == 5 and np.array_equal(nol[0][1].indices, golden["ref_part_indices"][ptr[0]:ptr[1]])


def test_map_function_matches_reference(golden):
    A = golden_csr(golden, "A_kdd_vals")[:40]
    R = golden_R(golden, 1)
    ptr = golden["ref_map_indptr"]
    for i in range(40):
        s, e = A.indptr[i], A.indptr[i + 1]
        v = random_project_map_function(SparseVector(A.shape[1], A.indices[s:e], A.data[s:e].astype(np.float64)), R)
        assert np.array_equal(v.indices, golden["ref_map_indices"][ptr[i]:ptr[i + 1]])
        assert same_bits(v.values, golden["ref_map_values"][ptr[i]:ptr[i + 1]])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("container", ["csr_matrix", "csr_array"])
def test_sklearn_transform_bitwise(dtype, container):
    from sklearn.random_projection import SparseRandomProjection as SkSRP
    from randomprojection_amd import SparseRandomProjection

    rng = np.random.default_rng(1)
    m = 50_000
    X = kdd_like(rng, 3000, m, values="normal", dtype=dtype)
    if container == "csr_array":
        X = sp.csr_array(X)
    ours = SparseRandomProjection(n_components=512, random_state=123).fit(X)
    ref = SkSRP(n_components=512, random_state=123).fit(X)
    assert same_bits(ours.components_.data, ref.components_.data)
    Y, Yr = ours.transform(X), ref.transform(X)
    assert type(Y) is type(Yr) and Y.dtype == Yr.dtype and Y.indices.dtype == Yr.indices.dtype
    assert_same_csr(Y, Yr.indptr, Yr.indices, Yr.data)
    ours.dense_output = True
    ref.dense_output = True
    assert same_bits(ours.transform(X), ref.transform(X))


def test_sklearn_refit_and_inplace_edit_reupload():
    """fit, transform, refit (other seed), transform: the second transform uses the new matrix
    (the cached GPU copy of R is keyed by the matrix object itself, never by a reusable id);
    an in-place edit of components_ is picked up as well."""
    from sklearn.random_projection import SparseRandomProjection as SkSRP
    from randomprojection_amd import SparseRandomProjection

    rng = np.random.default_rng(2)
    X = kdd_like(rng, 2000, 20_000, values="normal")
    ours = SparseRandomProjection(n_components=256, random_state=1).fit(X)
    Y1 = ours.transform(X)
    for seed in (2, 3, 1):
        ours.set_params(random_state=seed).fit(X)
        ref = SkSRP(n_components=256, random_state=seed).fit(X)
        Yr = ref.transform(X)
        Y = ours.transform(X)
        assert_same_csr(Y, Yr.indptr, Yr.indices, Yr.data)
        if seed != 1:
            assert (Y != Y1).nnz > 0
    ours.components_.data[:] = -ours.components_.data   # in place: same object, new values
    Y = ours.transform(X)
    assert same_bits(Y.data, -Y1.data) and np.array_equal(Y.indices, Y1.indices)


@pytest.mark.parametrize("powerlaw", [False, True])
@pytest.mark.parametrize("layout", ["auto", "generic"])
def test_random_kdd_shape_vs_oracle(powerlaw, layout):
    rng = np.random.default_rng(7 + powerlaw)
    m, p = 2_000_000, 4096
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = kdd_like(rng, 100_000, m, powerlaw=powerlaw, values="normal")
    P = Projector(R, layout=layout)
    C = P.matmul(A)
    assert_same_csr(C, *oracle_product(A, R))


def test_cfg4_shape_vs_oracle():
    """config 4 shape (100 nnz/row power-law, p=1024), scaled to m=2M."""
    rng = np.random.default_rng(4)
    m, p = 2_000_000, 1024
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    A = kdd_like(rng, 5000, m, mean=99, powerlaw=True, values="normal")
    C = Projector(R).matmul(A)
    assert_same_csr(C, *oracle_product(A, R))


def test_long_rows_and_heavy_tiles():
    """Rows beyond the LDS caps (tile > 4096 entries, row > 192 products) take the exact
    sequential path; results stay bit-identical."""
    rng = np.random.default_rng(11)
    m, p = 5000, 64
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123), dtype=np.float64)
    parts = [kdd_like(rng, 50, m, mean=10, values="normal", dtype=np.float64),
             kdd_like(rng, 3, m, mean=900, values="normal", dtype=np.float64, cap=m),
             kdd_like(rng, 20, m, mean=300, values="normal", dtype=np.float64),
             kdd_like(rng, 400, m, mean=3, values="normal", dtype=np.float64)]
    A = sp.vstack(parts).tocsr()
    for order in ("scipy", "sorted"):
        C = Projector(R).matmul(A, order=order)
        Cp, Cj, Cx = oracle_product(A, R)
        if order == "sorted":
            Cj, Cx = smmp.sorted_rows(Cp, Cj, Cx)
        assert_same_csr(C, Cp, Cj, Cx)


def test_empty_inputs():
    R = sm.projection_operand(sm.sparse_random_matrix(32, 1000, random_state=123))
    P = Projector(R)
    C = P.matmul(sp.csr_matrix((0, 1000), dtype=np.float32))
    assert C.shape == (0, 32) and C.nnz == 0
    C = P.matmul(sp.csr_matrix((17, 1000), dtype=np.float32))
    assert C.shape == (17, 32) and C.nnz == 0 and np.all(C.indptr == 0)


def test_errors_are_loud():
    R = sm.projection_operand(sm.sparse_random_matrix(32, 1000, random_state=123))
    P = Projector(R)
    with pytest.raises(ValueError, match="dimension mismatch"):
        P.matmul(sp.csr_matrix((3, 999), dtype=np.float32))
    bad = sp.csr_matrix((np.ones(1, np.float32), np.array([5000], np.int32), np.array([0, 1])), shape=(1, 1000))
    with pytest.raises(ValueError):
        P.matmul(bad)


def test_index64_inputs_follow_scipy_dtype_rule():
    """scipy picks int64 output indices for int64 inputs, then the container's constructor decides:
    csr_matrix downcasts indices that fit (int32), csr_array keeps int64. Same here."""
    rng = np.random.default_rng(3)
    m = 20_000
    R = sm.projection_operand(sm.sparse_random_matrix(128, m, random_state=123))
    A = kdd_like(rng, 500, m, values="normal")
    P = Projector(R)
    for cls, want in ((sp.csr_array, np.int64), (sp.csr_matrix, np.int32)):
        A64 = cls((A.data, A.indices.astype(np.int64), A.indptr.astype(np.int64)), shape=A.shape)
        if cls is sp.csr_matrix:
            A64.indices = A64.indices.astype(np.int64)
            A64.indptr = A64.indptr.astype(np.int64)
        C, Cr = P.matmul(A64), A64 @ R
        assert type(C) is type(Cr)
        assert C.indices.dtype == Cr.indices.dtype == want and C.indptr.dtype == Cr.indptr.dtype
        assert_same_csr(C, Cr.indptr, Cr.indices, Cr.data)


@pytest.mark.parametrize("threads", ["4", "0"])
def test_large_host_fetch_pipelined(threads):
    """Outputs past 16 MB are downloaded in chunks while helper threads pre-fault the fresh numpy
    destinations (option host_threads=0: plain copies); every index/value dtype combination."""
    rng = np.random.default_rng(21)
    m, p, n = 2_000_000, 4096, 1_500_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    k = 1 + rng.poisson(10, size=n)
    indptr = np.concatenate([[0], np.cumsum(k)]).astype(np.int64)
    idx = rng.integers(0, m, size=int(indptr[-1])).astype(np.int32)
    val = rng.standard_normal(idx.size).astype(np.float32)
    A = sp.csr_matrix((val, idx, indptr), shape=(n, m))
    Cp, Cj, Cx = oracle_product(A, R)
    assert Cj.size * 8 > (16 << 20)
    P = Projector(R)
    P.set_option("host_threads", int(threads))  # 4 = the default
    for dt in (np.int32, np.int64):
        ip, ix, dx = P.project_arrays(A.indptr, A.indices, A.data, out_index_dtype=dt)
        assert ip.dtype == ix.dtype == dt
        assert np.array_equal(ip, Cp) and np.array_equal(ix, Cj) and same_bits(dx, Cx)
    ip, ix, dx = P.project_arrays(A.indptr, A.indices, A.data.astype(np.float64))
    # (A.astype would canonicalise A's unsorted, duplicated rows: build the f64 twin from the arrays)
    C64 = oracle_product(sp.csr_matrix((A.data.astype(np.float64), A.indices, A.indptr), shape=A.shape), R)
    assert np.array_equal(ip, C64[0]) and np.array_equal(ix, C64[1]) and same_bits(dx, C64[2])


@pytest.mark.slow
def test_full_kdd_R_vs_oracle():
    """The recipe's own R (54,686,452 x 4096, random_state=123) on 60k KDD-shaped rows."""
    C0 = sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123)
    R = sm.projection_operand(C0)
    assert sm.csr_digest(R.indptr, R.indices, R.data) == sm.KDD_R_CSR_DIGEST
    P = Projector(R)
    assert P.layout == "packed" and P.nnz == 30_302_336
    rng = np.random.default_rng(2012)
    for powerlaw in (False, True):
        A = kdd_like(rng, 60_000, sm.KDD_M, powerlaw=powerlaw)
        assert_same_csr(P.matmul(A), *oracle_product(A, R))


def test_device_path_torch_and_capacity():
    import torch
    from randomprojection_amd import _native as nat

    m, p = 1_000_000, 4096
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    rng = np.random.default_rng(5)
    A = kdd_like(rng, 20_000, m, values="normal")
    dev = torch.device("cuda", 0)
    for ip_t, op_t, oi_t in [(torch.int32, torch.int32, torch.int32), (torch.int64, torch.int64, torch.int64),
                             (torch.int32, torch.int64, torch.int32)]:
        Ap = torch.as_tensor(A.indptr.astype(np.int64)).to(dev, ip_t)
        Aj = torch.as_tensor(A.indices).to(dev)
        Ax = torch.as_tensor(A.data).to(dev)
        Cp = torch.empty(A.shape[0] + 1, dtype=op_t, device=dev)
        small_j = torch.empty(10, dtype=oi_t, device=dev)
        small_x = torch.empty(10, dtype=torch.float32, device=dev)
        with pytest.raises(nat.RPError) as ei:
            P.project_device(Ap, Aj, Ax, Cp, small_j, small_x)
        nnz = ei.value.nnz
        Cj = torch.empty(nnz, dtype=oi_t, device=dev)
        Cx = torch.empty(nnz, dtype=torch.float32, device=dev)
        assert P.project_device(Ap, Aj, Ax, Cp, Cj, Cx) == nnz
        torch.cuda.synchronize()
        assert_same_csr(sp.csr_matrix((Cx.cpu().numpy(), Cj.cpu().numpy(), Cp.cpu().numpy()), shape=(A.shape[0], p)),
                        *oracle_product(A, R))


def test_projector_image_roundtrip():
    import torch

    R = sm.projection_operand(sm.sparse_random_matrix(256, 100_000, random_state=123))
    P = Projector(R)
    bufs = [torch.empty(max(b, 1), dtype=torch.uint8, device="cuda:0") for b in P.image_nbytes()]
    P.export_image([b.data_ptr() for b in bufs])
    Q = Projector.from_image(P.info, [b.data_ptr() for b in bufs], device=0)
    A = kdd_like(np.random.default_rng(9), 2000, 100_000, values="normal")
    C1, C2 = P.matmul(A), Q.matmul(A)
    assert_same_csr(C1, C2.indptr, C2.indices, C2.data)


def test_synthetic_rows_generator():
    import torch
    from randomprojection_amd import synth

    for dist in ("uniform", "powerlaw"):
        Ap, Aj, Ax = synth.kdd_rows_device(200_000, sm.KDD_M, seed=3, dist=dist, device=0)
        ap = Ap.cpu().numpy().astype(np.int64)
        aj = Aj.cpu().numpy()
        assert ap[0] == 0 and np.all(np.diff(ap) >= 1)
        assert 10.5 < ap[-1] / 200_000 < 11.5
        assert aj.min() >= 0 and aj.max() < sm.KDD_M
        rows = np.repeat(np.arange(200_000), np.diff(ap))
        d = np.diff(aj.astype(np.int64))
        same_row = rows[1:] == rows[:-1]
        assert np.all(d[same_row] > 0)              # strictly increasing inside rows
        assert torch.all(Ax == 1.0)
