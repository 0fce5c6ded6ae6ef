"""Dense Gaussian random projection on the MI355X (BASELINE.json configs[4]).

Reference semantics: sklearn ``GaussianRandomProjection`` — ``components_ = rng.normal(0,
1/sqrt(p), (p, m))`` (sklearn/random_projection.py:169-206, cast to X's dtype at fit) and
``transform(X) = X @ components_.T`` (:569-612), a plain dense GEMM (n x m) . (m x p). The
reference scripts never call it; BASELINE lists it as the dense-contraction config.

This module streams X through the GPU in row chunks and runs librp's hand-written MFMA GEMMs
(csrc/rp_dense.hip, ``rp_dense_project_device``) in
  * "fp32": f32 inputs, f32 MFMA (exact f32 products; gfx950 has no xf32) with f32 accumulation —
    matches numpy's sgemm within summation-order rounding (normwise 1e-5);
  * "fp64": f64 inputs, v_mfma_f64_16x16x4_f64 with f64 accumulation (sklearn computes in X's dtype);
  * "bf16": inputs rounded to bf16, f32 accumulation (2x less HBM, 16x the f32 MFMA rate) —
    documented reduced-precision mode, checked against an fp64 product of the bf16-rounded inputs.
The kernels are the product path for device-resident X too, a deliberate trade-off (hand-written
MFMA path, no library GEMM on the shipped path): on the same 131072 x 16384 -> 1024 block the
four-stage ring kernel measured bf16 1114 TF vs 1302 TF for hipBLASLt (0.86x) and f32 145 vs 154 TF
(0.94x), f64 58.8 vs 74.9 TF (profiles/r03_dense_*; scripts/bench_dense.py reports both per run).
End to end the configs[4] pass is PCIe-bound either way (X does not fit in HBM).
``components_`` is generated bit-identically to sklearn (``srp_matrix.gaussian_random_matrix``).
"""
from __future__ import annotations

import numpy as np
from sklearn.random_projection import GaussianRandomProjection as _SkGaussianRandomProjection
from sklearn.utils import check_random_state
from sklearn.utils.validation import check_is_fitted, validate_data

from .srp_matrix import gaussian_random_matrix

__all__ = ["GaussianRandomProjection", "dense_project_device", "prepare_operand"]


def _torch():
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError("GaussianRandomProjection.transform needs an MI355X (no CPU fallback)")
    return torch


_STEP = {"bf16": 64, "fp32": 32, "fp64": 16}  # K multiple each kernel needs (zeros are padded)


def _dtype(torch, compute):
    try:
        return {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[compute]
    except KeyError:
        raise ValueError("compute must be 'fp32', 'fp64' or 'bf16'") from None


def prepare_operand(A, compute: str):
    """A (rows x m) cast to the compute dtype, contiguous, the contraction padded with zeros to the
    kernel's K multiple (zeros add nothing). Done once for the components in ``transform``."""
    torch = _torch()
    A = A.to(_dtype(torch, compute)).contiguous()
    step = _STEP[compute]
    if A.shape[1] % step:
        A = torch.nn.functional.pad(A, (0, step - A.shape[1] % step))
    return A


def dense_project_device(X, C, out=None, compute: str = "fp32", stream=None, prepared_c: bool = False,
                         variant: int = -1):
    """``X @ C.T`` for device tensors X (n x m) and C (p x m) on librp's MFMA GEMM
    (rp_dense_project_device): "fp32" (exact-f32 MFMA, f32 result), "bf16" (bf16 inputs, f32
    accumulate, f32 result) or "fp64" (f64 MFMA, f64 result). ``prepared_c``: C already went through
    ``prepare_operand`` for this compute mode. ``variant``: -1 the default kernel, 0..11 another
    measured tile variant for this call only. Runs on ``stream`` (default: torch's current stream);
    temporaries made here are tied to that stream, so the caching allocator never hands them out
    while the GEMM may still read them."""
    import ctypes

    from . import _native as nat

    torch = _torch()
    Cc = C if prepared_c else prepare_operand(C, compute)
    n, m = X.shape
    p = Cc.shape[0]
    step = _STEP[compute]
    if Cc.shape[1] != (m + step - 1) // step * step:
        raise ValueError(f"matmul: dimension mismatch {tuple(X.shape)} @ {tuple(C.shape)}.T")
    Xc = prepare_operand(X, compute)
    ydt = torch.float64 if compute == "fp64" else torch.float32
    y = out if out is not None else torch.empty(n, p, dtype=ydt, device=X.device)
    if y.dtype != ydt or y.shape != (n, p) or y.stride(1) != 1:
        raise ValueError(f"out must be a {ydt} (n, p) tensor with unit column stride")
    cur = torch.cuda.current_stream(X.device)
    if stream is None:
        stream = cur.cuda_stream
    elif stream != cur.cuda_stream:
        # the GEMM reads Xc / Cc on another stream: order it after the casts / pads queued on the
        # current stream (an event wait on the device, no host sync), and keep them alive for it
        ext = torch.cuda.ExternalStream(stream, device=X.device)
        ext.wait_stream(cur)
        for t in (Xc, Cc):
            t.record_stream(ext)
    code = {"bf16": nat.RP_BF16, "fp32": nat.RP_F32, "fp64": nat.RP_F64}[compute]
    nat.check(nat.load().rp_dense_project_device(
        X.device.index or 0, ctypes.c_void_p(Xc.data_ptr()), code, n, Xc.shape[1], ctypes.c_void_p(Cc.data_ptr()), p,
        ctypes.c_void_p(y.data_ptr()), y.stride(0), ctypes.c_void_p(stream), int(variant)))
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
        Cp = prepare_operand(C, mode)  # cast and padded once for every chunk
        n = X.shape[0]
        out = np.empty((n, C.shape[0]), dtype=wdt)
        for s in range(0, n, self.chunk_rows):
            e = min(n, s + self.chunk_rows)
            blk = X[s:e]
            blk = blk.toarray() if sp.issparse(blk) else blk
            xb = torch.as_tensor(np.ascontiguousarray(blk, dtype=wdt), device=dev)
            out[s:e] = dense_project_device(xb, Cp, compute=mode, prepared_c=True).cpu().numpy()
        return out

    def __getstate__(self):
        return self.__dict__.copy()
