"""BASELINE.json configs at their real sizes on one MI355X (device-resident path):

* configs[1]: all 119,705,032 KDD2012-shaped rows x 54,686,452 -> 4096 (uniform and power-law
  columns, scipy and sorted row order), device-resident and streamed from host memory;
* configs[2]: all 1,077,345,288 rows (9x KDD2012) on ONE GPU — output nnz > 2^31, so int64
  output indptr;
* configs[3]: power-law rows with exactly 100 nnz over the real m = 10,000,000 features -> 1024,
  at its full 200,000,000 rows in one call (2.0e10 input entries, 6.3e9 output entries: int64
  input and output indptr, entries stored past 2^31 and 2^32), and at 4M rows in both orders.

Whole outputs are checked on the device (indptr from 0 to nnz and monotone, columns in [0, p),
rows ascending for the sorted order); >= 64k rows spread over the matrix (plus the last rows, past
2^31 output entries for configs[2]) are compared bit for bit with the oracle's restatement of
scipy's csr_matmat (reference path: code/clustermode/randomProjection.py:46 -> scipy csr_matmat).
"""
import gc

import numpy as np
import pytest

from gpu_helpers import check_csr_on_device, check_rows_vs_oracle, sample_rows
from randomprojection_amd import Projector, srp_matrix as sm, synth
from randomprojection_amd import _native as nat

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

KDD_ROWS = 119_705_032


@pytest.fixture(scope="module")
def kdd():
    import torch

    torch.cuda.empty_cache()
    R = sm.projection_operand(sm.sparse_random_matrix(sm.KDD_P, sm.KDD_M, random_state=123))
    assert sm.csr_digest(R.indptr, R.indices, R.data) == sm.KDD_R_CSR_DIGEST
    P = Projector(R)
    assert P.layout == "packed" and P.nnz == 30_302_336
    yield R, P
    P.close()
    torch.cuda.empty_cache()


def project(P, Ap, Aj, Ax, order="scipy", slack=1.02):
    """Device product into freshly sized outputs (int64 indptr once the estimate passes 2^31);
    one exact retry if the estimate was short."""
    import torch

    dev = Aj.device
    n = Ap.numel() - 1
    nnz_a = int(Aj.numel())
    ws_bytes = P.workspace_bytes(n, nnz_a, dtype=Ax.dtype)
    cap = int(slack * nnz_a * P.nnz / P.m) + 65536
    # the HBM budget, stated before anything is allocated: workspace + C (indptr, indices, values)
    # must fit next to A in what the device has free; a shortfall is named, not an opaque OOM
    c_bytes = (n + 1) * (8 if cap >= 2**31 else 4) + cap * (4 + Ax.element_size())
    free, total = torch.cuda.mem_get_info(dev)
    need = ws_bytes + c_bytes
    assert need <= free - (1 << 30), (
        f"HBM budget: workspace {ws_bytes / 2**30:.1f} GiB + C {c_bytes / 2**30:.1f} GiB = {need / 2**30:.1f} GiB "
        f"> {free / 2**30:.1f} GiB free of {total / 2**30:.1f} GiB (A holds {torch.cuda.memory_allocated(dev) / 2**30:.1f} "
        "GiB); 1 GiB kept for the allocator")
    print(f"HBM budget: workspace {ws_bytes / 2**30:.1f} + C {c_bytes / 2**30:.1f} of {free / 2**30:.1f} GiB free")
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    for _ in range(2):
        Cp = torch.empty(n + 1, dtype=torch.int64 if cap >= 2**31 else torch.int32, device=dev)
        Cj = torch.empty(cap, dtype=torch.int32, device=dev)
        Cx = torch.empty(cap, dtype=torch.float32, device=dev)
        try:
            nnz = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=order, workspace=ws, nnz_a=nnz_a)
            project.staged = P.choice(n, nnz_a, ws)  # what the device chose (auto mode)
            return Cp, Cj, Cx, nnz
        except nat.RPError as e:
            if e.code != nat.RP_ERR_CAPACITY:
                raise
            cap = e.nnz
        del Cp, Cj, Cx  # before the exact retry allocates again (full-size outputs are tens of GB)
        gc.collect()
    raise AssertionError("capacity retry failed")


@pytest.mark.parametrize("dist", ["uniform", "powerlaw"])
def test_configs1_full_size(kdd, dist, monkeypatch):
    import torch

    R, P = kdd
    Ap, Aj, Ax = synth.kdd_rows_device(KDD_ROWS, sm.KDD_M, seed=2012 if dist == "uniform" else 2013, dist=dist)
    assert 10.9 < Aj.numel() / KDD_ROWS < 11.1
    rows = sample_rows(KDD_ROWS, 65536)
    orders = ("scipy", "sorted") if dist == "uniform" else ("scipy",)
    for order in orders:
        Cp, Cj, Cx, nnz = project(P, Ap, Aj, Ax, order=order)
        assert 5.3 < nnz / KDD_ROWS < 6.3
        check_csr_on_device(Cp, Cj, nnz, sm.KDD_P, sorted_rows=(order == "sorted"))
        assert check_rows_vs_oracle(rows, Ap, Aj, Ax, Cp, Cj, Cx, R, order=order) > 350_000
        if order == "scipy":
            # the whole output against the other pipeline (the tile kernel with direct gathers):
            # every byte equal, so a rare tile shape mishandled by either one cannot hide between
            # the sampled rows
            assert P.plan(KDD_ROWS, Aj.numel()) == {"pipeline": "rowlane", "staged": "auto", "bucket_shift": 19}
            # the device's choice: staged gathers for uniform columns (each gather a fresh line),
            # direct for power-law ones (hot features stay in L2)
            assert project.staged == (dist == "uniform")
            P.set_option("pipeline", "tile")
            P.set_staging("off")
            Tp, Tj, Tx, tn = project(P, Ap, Aj, Ax, order=order)
            P.set_option("pipeline", None)
            P.set_staging("auto")
            assert tn == nnz and bool(torch.equal(Tp, Cp))
            for s in range(0, nnz, 1 << 28):
                e = min(nnz, s + (1 << 28))
                assert bool(torch.equal(Tj[s:e], Cj[s:e])) and bool(torch.equal(Tx[s:e].view(torch.int32),
                                                                                Cx[s:e].view(torch.int32)))
            del Tp, Tj, Tx
        if order == "scipy":
            # the same rows as a host CSR through the chunked stream path (boundary 2): the whole
            # 119.7M-row result equals the device-resident one, every byte; no chunk outgrew its
            # device slot (power-law columns give ~4% more outputs per entry than R's mean row
            # length predicts: round 5 recomputed every such chunk serially, 76 M rows/s)
            ip, ix, dx = P.project_stream(Ap.cpu().numpy(), Aj.cpu().numpy(), Ax.cpu().numpy())
            st = P.stream_stats()
            assert st["chunks"] == (KDD_ROWS + (2 << 20) - 1) // (2 << 20) and st["recomputed"] == 0, st
            assert ix.size == nnz
            assert np.array_equal(ip, Cp.cpu().numpy())
            assert np.array_equal(ix, Cj[:nnz].cpu().numpy())
            assert np.array_equal(dx.view(np.uint32), Cx[:nnz].cpu().numpy().view(np.uint32))
            del ip, ix, dx
        del Cp, Cj, Cx
        torch.cuda.empty_cache()


def test_configs2_full_size_one_gpu(kdd):
    """1,077,345,288 rows (~95 GB of A, ~53 GB of C) in one call on one MI355X."""
    import torch

    R, P = kdd
    n = 9 * KDD_ROWS
    torch.cuda.empty_cache()
    Ap, Aj, Ax = synth.kdd_rows_device(n, sm.KDD_M, seed=2021, indptr_dtype=torch.int64)
    assert Ap.dtype == torch.int64 and Aj.numel() > 2**33
    Cp, Cj, Cx, nnz = project(P, Ap, Aj, Ax)
    assert nnz > 2**32 and Cp.dtype == torch.int64
    check_csr_on_device(Cp, Cj, nnz, sm.KDD_P)
    rows = sample_rows(n, 65536)
    past = int((Cp[torch.as_tensor(rows, device=Cp.device)] > 2**31).sum().item())
    assert past > 30_000, "the sample must reach rows stored past 2^31 output entries"
    assert check_rows_vs_oracle(rows, Ap, Aj, Ax, Cp, Cj, Cx, R) > 350_000
    del Ap, Aj, Ax, Cp, Cj, Cx
    torch.cuda.empty_cache()


def test_configs3_real_m():
    """configs[3] shape at its real feature count: Zipf(1.1) power-law columns, exactly 100 distinct
    nnz per row, m = 10,000,000 -> p = 1024."""
    import torch

    torch.cuda.empty_cache()
    m, p, n = 10_000_000, 1024, 4_000_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    Ap, Aj, Ax = synth.kdd_rows_device(n, m, seed=4, dist="powerlaw", mean_extra=-100.0)
    assert Aj.numel() == 100 * n
    for order in ("scipy", "sorted"):
        Cp, Cj, Cx, nnz = project(P, Ap, Aj, Ax, order=order, slack=1.0)
        assert 25 < nnz / n < 40
        check_csr_on_device(Cp, Cj, nnz, p, sorted_rows=(order == "sorted"))
        assert check_rows_vs_oracle(sample_rows(n, 65536), Ap, Aj, Ax, Cp, Cj, Cx, R, order=order) > 1_000_000
        del Cp, Cj, Cx
    P.close()
    torch.cuda.empty_cache()


def test_configs3_full_size():
    """BASELINE configs[3] at its real size: 200,000,000 power-law rows x 10,000,000, exactly 100
    nnz per row -> 1024, one rp_project_device call on the tile pipeline with int64 input and output
    indptr (2.0e10 input entries, ~6.3e9 output entries). Whole output checked on the device in
    bounded chunks; >= 64k sampled rows bit-exact against the oracle, including rows stored past
    2^31 and past 2^32 output entries."""
    import gc

    import torch

    gc.collect()
    torch.cuda.empty_cache()
    print("before configs[3]: free/total", torch.cuda.mem_get_info(), "allocated", torch.cuda.memory_allocated())
    m, p, n = 10_000_000, 1024, 200_000_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    Ap, Aj, Ax = synth.kdd_rows_device(n, m, seed=5, dist="powerlaw", mean_extra=-100.0, indptr_dtype=torch.int64)
    assert Ap.dtype == torch.int64 and Aj.numel() == 100 * n
    assert P.plan(n, Aj.numel())["pipeline"] == "tile"
    print("A ready: allocated", torch.cuda.memory_allocated(), "workspace",
          P.workspace_bytes(n, Aj.numel(), dtype=Ax.dtype), P.workspace_bytes(n, Aj.numel()))
    Cp, Cj, Cx, nnz = project(P, Ap, Aj, Ax, slack=1.0)
    assert Cp.dtype == torch.int64 and nnz > 2**32 and 28 < nnz / n < 36
    check_csr_on_device(Cp, Cj, nnz, p)
    rows = sample_rows(n, 65536)
    off = Cp[torch.as_tensor(rows, device=Cp.device)]
    assert int((off > 2**31).sum().item()) > 40_000 and int((off > 2**32).sum().item()) > 15_000, \
        "the sample must reach rows stored past 2^31 and 2^32 output entries"
    assert check_rows_vs_oracle(rows, Ap, Aj, Ax, Cp, Cj, Cx, R) > 2_000_000
    del Ap, Aj, Ax, Cp, Cj, Cx
    P.close()
    torch.cuda.empty_cache()
