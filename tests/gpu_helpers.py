"""Whole-output property checks on the device and sampled bit-exact checks against the oracle, for
outputs too large to compare whole (BASELINE configs at full size). Test infrastructure only."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from oracle import smmp


def check_csr_on_device(Cp, Cj, nnz: int, p: int, sorted_rows: bool = False) -> None:
    """indptr starts at 0, ends at nnz and never decreases; every column in [0, p); with
    ``sorted_rows`` every row strictly ascending. All reductions run on the device."""
    import torch

    cp = Cp.to(torch.int64) if Cp.dtype != torch.int64 else Cp
    assert int(cp[0].item()) == 0, "indptr[0] != 0"
    assert int(cp[-1].item()) == nnz, f"indptr[-1] {int(cp[-1].item())} != nnz {nnz}"
    step = 1 << 28  # bounded temporaries on the largest outputs
    n = cp.numel() - 1
    for s in range(0, n, step):
        e = min(n, s + step)
        assert bool(torch.all(cp[s + 1:e + 1] >= cp[s:e]).item()), f"indptr decreases in rows [{s}, {e})"
    for s in range(0, nnz, step):
        c = Cj[s:min(nnz, s + step)]
        assert int(c.min().item()) >= 0 and int(c.max().item()) < p, "column out of range"
    if sorted_rows and nnz > 1:
        # an entry may be <= its predecessor only at a row start
        starts = torch.zeros(nnz + 1, dtype=torch.bool, device=Cj.device)
        starts[cp[:-1]] = True
        for s in range(1, nnz, step):
            e = min(nnz, s + step)
            ok = (Cj[s:e] > Cj[s - 1:e - 1]) | starts[s:e]
            assert bool(torch.all(ok).item()), "a row is not strictly ascending"


def sample_rows(n_rows: int, k: int, seed: int = 20261016, tail: int = 512) -> np.ndarray:
    """k distinct rows spread over the whole matrix, plus the last ``tail`` rows."""
    rng = np.random.default_rng(seed)
    k = min(k, n_rows)
    rows = rng.choice(n_rows, size=k, replace=False)
    rows = np.union1d(rows, np.arange(max(0, n_rows - tail), n_rows))
    return rows.astype(np.int64)


def gather_segments(t, lo, hi):
    """Device array segments [lo_i, hi_i) concatenated, gathered on the device, to numpy."""
    import torch

    lens = (hi - lo).astype(np.int64)
    if lens.sum() == 0:
        return t[:0].cpu().numpy()
    starts = np.repeat(lo - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
    idx = np.arange(int(lens.sum()), dtype=np.int64) + starts
    return t[torch.as_tensor(idx, device=t.device)].cpu().numpy()


def check_rows_vs_oracle(rows, Ap, Aj, Ax, Cp, Cj, Cx, R_host, order: str = "scipy") -> int:
    """The output rows ``rows`` equal the oracle's restatement of scipy's csr_matmat on the same
    input rows, bit for bit (indices in scipy's per-row order, or ascending for "sorted").
    Returns the number of output entries compared."""
    import torch

    r_t = torch.as_tensor(rows, device=Ap.device)
    s0 = Ap[r_t].to(torch.int64).cpu().numpy()
    s1 = Ap[r_t + 1].to(torch.int64).cpu().numpy()
    cp = Cp.to(torch.int64) if Cp.dtype != torch.int64 else Cp
    c0, c1 = cp[r_t].cpu().numpy(), cp[r_t + 1].cpu().numpy()
    ptr = np.concatenate([[0], np.cumsum(s1 - s0)])
    A = sp.csr_matrix((gather_segments(Ax, s0, s1), gather_segments(Aj, s0, s1), ptr),
                      shape=(rows.size, R_host.shape[0]))
    Wp, Wj, Wx, _, _ = smmp.matmat(A, R_host)
    if order == "sorted":
        Wj, Wx = smmp.sorted_rows(Wp, Wj, Wx)
    got_ptr = np.concatenate([[0], np.cumsum(c1 - c0)])
    assert np.array_equal(got_ptr, Wp), "row lengths differ from the oracle"
    gj, gx = gather_segments(Cj, c0, c1), gather_segments(Cx, c0, c1)
    assert np.array_equal(gj.astype(np.int64), Wj.astype(np.int64)), "indices differ from the oracle"
    assert np.array_equal(gx.view(np.uint32 if gx.dtype == np.float32 else np.uint64),
                          Wx.view(np.uint32 if Wx.dtype == np.float32 else np.uint64)), "value bits differ"
    return int(Wj.size)
