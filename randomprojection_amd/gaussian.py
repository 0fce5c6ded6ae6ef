"""Dense Gaussian random projection on the MI355X (BASELINE.json configs[4]).

Reference semantics: sklearn ``GaussianRandomProjection`` — ``components_ = rng.normal(0,
1/sqrt(p), (p, m))`` (sklearn/random_projection.py:169-206, cast to X's dtype at fit) and
``transform(X) = X @ components_.T`` (:569-612), a plain dense GEMM (n x m) . (m x p). The
reference scripts never call it; BASELINE lists it as the dense-contraction config.

This module streams X through the GPU in row chunks and runs librp's hand-written MFMA GEMM
(csrc/rp_dense.hip, ``rp_dense_project_device``) in
  * "fp32": f32 inputs, f32 MFMA (v_mfma_f32_32x32x2_f32 — exact f32 products; gfx950 has no xf32)
    with f32 accumulation — matches numpy's sgemm within summation-order rounding (normwise 1e-5);
  * "bf16": inputs rounded to bf16, f32 accumulation (v_mfma_f32_32x32x16_bf16; 2x less HBM, 16x
    MFMA rate) — documented reduced-precision mode, checked against an fp64 product of the
    bf16-rounded inputs.
f64 input (sklearn computes in X's dtype) goes to torch's f64 matmul (library GEMM).
``components_`` is generated bit-identically to sklearn (``srp_matrix.gaussian_random_matrix``).
"""
from __future__ import annotations

import numpy as np
from sklearn.random_projection import GaussianRandomProjection as _SkGaussianRandomProjection
from sklearn.utils import check_random_state
from sklearn.utils.validation import check_is_fitted, validate_data

from .srp_matrix import gaussian_random_matrix

__all__ = ["GaussianRandomProjection", "dense_project_device"]


def _torch():
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError("GaussianRandomProjection.transform needs an MI355X (no CPU fallback)")
    return torch


def dense_project_device(X, C, out=None, compute: str = "fp32", stream=None):
    """``X @ C.T`` for device tensors X (n x m) and C (p x m).
    ``compute``: "fp32" (exact-f32 MFMA, f32 result) or "bf16" (bf16 inputs, f32 accumulate, f32
    result) run librp's hand-written MFMA GEMM (rp_dense_project_device); "fp64" (f64 MFMA, f64
    result) goes to torch's matmul."""
    torch = _torch()
    if compute in ("fp32", "bf16"):
        import ctypes

        from . import _native as nat

        dt = torch.bfloat16 if compute == "bf16" else torch.float32
        Xc = X.to(dt).contiguous()
        Cc = C.to(dt).contiguous()
        n, m = Xc.shape
        p = Cc.shape[0]
        if Cc.shape[1] != m:
            raise ValueError(f"matmul: dimension mismatch {tuple(X.shape)} @ {tuple(C.shape)}.T")
        y = out if out is not None else torch.empty(n, p, dtype=torch.float32, device=X.device)
        if y.dtype != torch.float32 or y.shape != (n, p) or y.stride(1) != 1:
            raise ValueError("out must be a float32 (n, p) tensor with unit column stride")
        step = 64 if compute == "bf16" else 32
        if m % step:  # pad the contraction (zeros add nothing)
            padm = (m + step - 1) // step * step
            Xc = torch.nn.functional.pad(Xc, (0, padm - m))
            Cc = torch.nn.functional.pad(Cc, (0, padm - m))
            m = padm
        if stream is None:
            stream = torch.cuda.current_stream(X.device).cuda_stream
        nat.check(nat.load().rp_dense_project_device(
            X.device.index or 0, ctypes.c_void_p(Xc.data_ptr()), nat.RP_BF16 if compute == "bf16" else nat.RP_F32,
            n, m, ctypes.c_void_p(Cc.data_ptr()), p, ctypes.c_void_p(y.data_ptr()), y.stride(0),
            ctypes.c_void_p(stream)))
        return y
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False  # never a reduced-precision f32 path
    try:
        if compute == "bf16":
            Xb = X if X.dtype == torch.bfloat16 else X.to(torch.bfloat16)
            Cb = C if C.dtype == torch.bfloat16 else C.to(torch.bfloat16)
            # aten::mm.dtype: bf16 operands, f32 accumulate, f32 result (never rounded to bf16)
            y = torch.mm(Xb, Cb.t(), out_dtype=torch.float32)
        elif compute == "fp32":
            y = torch.matmul(X.float(), C.float().t())
        elif compute == "fp64":
            y = torch.matmul(X.double(), C.double().t())
        else:
            raise ValueError("compute must be 'fp32', 'fp64' or 'bf16'")
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev
    if out is not None:
        out.copy_(y)
        return out
    return y


class GaussianRandomProjection(_SkGaussianRandomProjection):
    """sklearn ``GaussianRandomProjection`` with a GPU ``transform`` (librp's MFMA GEMM).

    Extra parameters: ``device`` (GPU ordinal), ``compute`` ("auto" = X's dtype as sklearn
    computes, or "bf16"), ``chunk_rows`` (rows of X per device GEMM; bounds device memory)."""

    def __init__(self, n_components="auto", *, eps=0.1, compute_inverse_components=False,
                 random_state=None, device=0, compute="auto", chunk_rows=65536):
        super().__init__(n_components=n_components, eps=eps,
                         compute_inverse_components=compute_inverse_components,
                         random_state=random_state)
        self.device = device
        self.compute = compute
        self.chunk_rows = chunk_rows

    def _make_random_matrix(self, n_components, n_features):
        random_state = check_random_state(self.random_state)
        return gaussian_random_matrix(n_components, n_features, random_state=random_state)

    def transform(self, X):
        check_is_fitted(self)
        X = validate_data(self, X, accept_sparse=["csr", "csc"], reset=False,
                          dtype=[np.float64, np.float32])
        torch = _torch()
        dev = torch.device("cuda", self.device)
        import scipy.sparse as sp

        mode = self.compute if self.compute != "auto" else ("fp64" if X.dtype == np.float64 else "fp32")
        wdt = np.float64 if mode == "fp64" else np.float32
        C = torch.as_tensor(np.ascontiguousarray(self.components_, dtype=wdt), device=dev)
        n = X.shape[0]
        out = np.empty((n, C.shape[0]), dtype=wdt)
        for s in range(0, n, self.chunk_rows):
            e = min(n, s + self.chunk_rows)
            blk = X[s:e]
            blk = blk.toarray() if sp.issparse(blk) else blk
            xb = torch.as_tensor(np.ascontiguousarray(blk, dtype=wdt), device=dev)
            out[s:e] = dense_project_device(xb, C, compute=mode).cpu().numpy()
        return out

    def __getstate__(self):
        return self.__dict__.copy()
