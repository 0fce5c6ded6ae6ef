"""Dense Gaussian projection (configs[4] path): GPU GEMM vs sklearn/numpy within the north-star
tolerance (normwise 1e-5 fp32, 1e-12 fp64), bf16 mode vs an fp64 product of bf16-rounded inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / np.linalg.norm(b.ravel()))


@pytest.mark.parametrize("dtype,tol", [(np.float32, 1e-5), (np.float64, 1e-12)])
def test_transform_matches_sklearn(dtype, tol):
    from sklearn.random_projection import GaussianRandomProjection as Sk
    from randomprojection_amd.gaussian import GaussianRandomProjection

    rng = np.random.default_rng(0)
    X = rng.standard_normal((3000, 16384)).astype(dtype)
    ours = GaussianRandomProjection(n_components=1024, random_state=123, chunk_rows=1000).fit(X)
    ref = Sk(n_components=1024, random_state=123).fit(X)
    assert np.array_equal(ours.components_, ref.components_)
    Y, Yr = ours.transform(X), ref.transform(X)
    assert Y.dtype == Yr.dtype and Y.shape == Yr.shape
    exact = X.astype(np.float64) @ ref.components_.astype(np.float64).T
    assert _rel(Y, exact) < tol and _rel(Y, Yr) < 2 * tol


def test_bf16_mode():
    import torch
    from randomprojection_amd.gaussian import dense_project_device

    rng = np.random.default_rng(1)
    X = torch.as_tensor(rng.standard_normal((4096, 16384)).astype(np.float32), device="cuda")
    C = torch.as_tensor(rng.normal(0, 1 / 32, (1024, 16384)).astype(np.float32), device="cuda")
    Y = dense_project_device(X, C, compute="bf16").cpu().numpy()
    Xb = X.to(torch.bfloat16).double().cpu().numpy()
    Cb = C.to(torch.bfloat16).double().cpu().numpy()
    assert _rel(Y, Xb @ Cb.T) < 1e-5


def test_sparse_input():
    import scipy.sparse as sp
    from sklearn.random_projection import GaussianRandomProjection as Sk
    from randomprojection_amd.gaussian import GaussianRandomProjection

    X = sp.random(500, 4000, density=0.01, format="csr", dtype=np.float32, random_state=2)
    ours = GaussianRandomProjection(n_components=256, random_state=7).fit(X)
    ref = Sk(n_components=256, random_state=7).fit(X)
    assert _rel(ours.transform(X), ref.transform(X)) < 1e-5


@pytest.mark.parametrize("variant", [-1, 5, 10, 11])
@pytest.mark.parametrize("compute", ["fp32", "bf16", "fp64"])
@pytest.mark.parametrize("shape", [(1, 64, 1), (300, 4096, 200), (1000, 16384, 1024), (257, 192, 129)])
def test_mfma_kernel_ragged_shapes(compute, shape, variant):
    """librp's MFMA GEMM kernels (the default, the register-staged 256 x 256 tile and the LDS-direct
    one) on ragged tiles (rows / columns past the block, m not a multiple of the K step: padded)
    against an fp64 product of the same (bf16-rounded) operands."""
    import torch
    from randomprojection_amd.gaussian import dense_project_device

    if compute == "fp64" and variant not in (-1, 10):
        pytest.skip("two f64 kernels: the ring (default) and the two-buffer one (variant 10)")

    n, m, p = shape
    rng = np.random.default_rng(n + m + p)
    wdt = np.float64 if compute == "fp64" else np.float32
    X = torch.as_tensor(rng.standard_normal((n, m)).astype(wdt), device="cuda")
    C = torch.as_tensor(rng.normal(0, 1 / 32, (p, m)).astype(wdt), device="cuda")
    Y = dense_project_device(X, C, compute=compute, variant=variant).cpu().numpy()
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[compute]
    ref = X.to(dt).double().cpu().numpy() @ C.to(dt).double().cpu().numpy().T
    assert Y.shape == (n, p) and Y.dtype == wdt
    # north_star tolerances: fp32 1e-5 (K = 16384 f32 fma chains: ~2e-6 measured), fp64 1e-12
    assert _rel(Y, ref) < (1e-12 if compute == "fp64" else 1e-5)
    out = torch.full((n, p + 7), 7.0, device="cuda", dtype=torch.float64 if compute == "fp64" else torch.float32)[:, :p]
    dense_project_device(X, C, out=out, compute=compute, variant=variant)
    assert np.array_equal(out.cpu().numpy(), Y)


@pytest.mark.parametrize("compute", ["bf16", "fp32"])
def test_side_stream_waits_for_casts(compute):
    """dense_project_device on a stream other than torch's current one, with operands that need a
    cast and a K pad (prepared on the current stream): the GEMM waits for them, so the
    result equals the current-stream run bit for bit."""
    import torch
    from randomprojection_amd.gaussian import dense_project_device

    rng = np.random.default_rng(11)
    X = torch.as_tensor(rng.standard_normal((5000, 4001)), device="cuda")  # f64 in, m not a K-step multiple
    C = torch.as_tensor(rng.normal(0, 1 / 32, (384, 4001)), device="cuda")
    want = dense_project_device(X, C, compute=compute)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    got = dense_project_device(X, C, compute=compute, stream=side.cuda_stream)
    side.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_configs4_width_million_rows(compute):
    """configs[4]'s full m x p (16384 -> 1024) on 1,000,003 device-resident rows (64 GB of f32 X;
    the 10M-row pass itself is 655 GB and streams from the host): ONE librp GEMM launch over every
    row, each 65,536-row block (the ragged last one included) against a chunked fp64 torch product
    of the same (bf16-rounded for "bf16") operands, normwise within the north-star 1e-5."""
    import torch
    from randomprojection_amd.gaussian import dense_project_device, prepare_operand

    n, m, p = 1_000_003, 16384, 1024
    g = torch.Generator(device="cuda").manual_seed(4)
    X = torch.randn(n, m, device="cuda", dtype=torch.float32, generator=g)
    C = torch.randn(p, m, device="cuda", dtype=torch.float32, generator=g) / 128.0
    Cc = prepare_operand(C, compute)
    Y = dense_project_device(X, Cc, compute=compute, prepared_c=True)
    assert Y.shape == (n, p) and Y.dtype == torch.float32
    dt = torch.bfloat16 if compute == "bf16" else torch.float32
    Cd = C.to(dt).double()
    worst = 0.0
    for s in range(0, n, 65536):
        e = min(n, s + 65536)
        ref = X[s:e].to(dt).double() @ Cd.T
        rel = float(torch.linalg.norm(Y[s:e].double() - ref) / torch.linalg.norm(ref))
        worst = max(worst, rel)
        del ref
    assert bool(torch.isfinite(Y).all()) and worst < 1e-5, worst
