"""The packed single-magnitude image of R (built on the host by rp_pack_r_host, the same code
rp_projector_create uploads) decodes back to R exactly: rows, per-row order, signs."""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp

from randomprojection_amd import _native as nat
from randomprojection_amd import srp_matrix as sm


def pack(R, layout=nat.RP_LAYOUT_AUTO):
    lib = nat.load()
    R = sp.csr_matrix(R)
    info = nat.ProjectorInfo()
    args = (R.shape[0], R.shape[1], nat.ptr(R.indptr), nat.idx_code(R.indptr.dtype), nat.ptr(R.indices),
            nat.idx_code(R.indices.dtype), nat.ptr(R.data), nat.val_code(R.data.dtype), layout, ctypes.byref(info))
    nat.check(lib.rp_pack_r_host(*args, None, None, None))
    bufs = [np.zeros(max(int(info.buffer_bytes[i]), 1), np.uint8) for i in range(3)]
    nat.check(lib.rp_pack_r_host(*args, *[nat.ptr(b) for b in bufs]))
    return info, bufs


def decode_packed(info, bufs, dtype):
    """Decode the 64-bit packed image: n = w >> 61 entries inline (15 bits each:
    sign << 14 | column), or n == 7: record at O[w & (2^61-1)] = count, (sign << 15 | column)..."""
    W = bufs[0][:info.buffer_bytes[0]].view(np.uint64)
    O = bufs[1][:info.buffer_bytes[1]].view(np.uint16)
    mag = dtype(info.magnitude)
    indptr, cols, vals = [0], [], []
    for w in W.tolist():
        n = w >> 61
        if n == 7:
            rec = w & ((1 << 61) - 1)
            k = int(O[rec])
            ent = O[rec + 1: rec + 1 + k].astype(np.int64)
            cols.extend((ent & 0x7FFF).tolist())
            vals.extend(np.where(ent & 0x8000, -mag, mag).tolist())
        else:
            assert w >> (15 * n) & ((1 << (61 - 15 * n)) - 1) == 0   # unused bits are clear
            for t in range(n):
                e = (w >> (15 * t)) & 0x7FFF
                cols.append(e & 0x3FFF)
                vals.append(-mag if e & 0x4000 else mag)
        indptr.append(len(cols))
    return np.array(indptr), np.array(cols), np.array(vals, dtype=dtype)


@pytest.mark.parametrize("m,p,dtype", [(100_000, 256, np.float32), (5000, 64, np.float64), (3000, 4096, np.float32)])
def test_packed_roundtrip(m, p, dtype):
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123), dtype=dtype)
    info, bufs = pack(R)
    assert info.layout == nat.RP_LAYOUT_PACKED and info.nnz == R.nnz
    assert info.magnitude == float(np.abs(R.data[0]))
    ip, ix, vx = decode_packed(info, bufs, dtype)
    assert np.array_equal(ip, R.indptr) and np.array_equal(ix, R.indices)
    assert np.array_equal(vx.view(np.uint8), R.data.view(np.uint8))
    assert info.buffer_bytes[0] == 8 * m                       # one u64 word per feature


def test_long_rows_use_records():
    """Features with more than 4 entries are stored as records; order and signs survive."""
    rng = np.random.default_rng(0)
    m, p = 3000, 16384
    k = rng.integers(0, 12, size=m)
    rows = [rng.choice(p, size=int(x), replace=False) for x in k]     # unsorted storage order
    indptr = np.concatenate([[0], np.cumsum(k)])
    R = sp.csr_matrix((np.where(rng.random(indptr[-1]) < .5, -2.5, 2.5).astype(np.float32),
                       np.concatenate(rows), indptr), shape=(m, p))
    info, bufs = pack(R)
    assert info.layout == nat.RP_LAYOUT_PACKED and info.buffer_bytes[1] > 0
    ip, ix, vx = decode_packed(info, bufs, np.float32)
    assert np.array_equal(ip, R.indptr) and np.array_equal(ix, R.indices) and np.array_equal(vx, R.data)


def test_generic_when_magnitudes_differ_or_forced():
    R = sp.random(2000, 64, density=0.02, format="csr", dtype=np.float32, random_state=1)
    info, bufs = pack(R)
    assert info.layout == nat.RP_LAYOUT_GENERIC
    Bp = bufs[0][:info.buffer_bytes[0]].view(np.int32)
    Bj = bufs[1][:info.buffer_bytes[1]].view(np.uint16)
    Bx = bufs[2][:info.buffer_bytes[2]].view(np.float32)
    assert np.array_equal(Bp, R.indptr) and np.array_equal(Bj, R.indices) and np.array_equal(Bx, R.data)
    R1 = sm.projection_operand(sm.sparse_random_matrix(64, 2000, random_state=123))
    assert pack(R1, nat.RP_LAYOUT_GENERIC)[0].layout == nat.RP_LAYOUT_GENERIC
    with pytest.raises(nat.RPError):
        pack(R, nat.RP_LAYOUT_PACKED)


def test_explicit_zero_entries_force_generic():
    R = sm.projection_operand(sm.sparse_random_matrix(32, 1000, random_state=123))
    R.data[3] = 0.0
    assert pack(R)[0].layout == nat.RP_LAYOUT_GENERIC


def test_invalid_r_rejected():
    R = sp.csr_matrix((np.ones(2, np.float32), np.array([0, 70]), np.array([0, 1, 2])), shape=(2, 64))
    with pytest.raises(nat.RPError, match="out of range"):
        pack(R)


def test_documented_shape_limits():
    """Limits scipy does not have, documented in DESIGN.md §7: p <= 32767 for any R on the GPU
    path, and the packed layout only for p <= 16384 (a 15-bit slot: sign << 14 | column) — a
    single-magnitude R with wider p falls back to the generic layout, and RP_LAYOUT_PACKED then
    refuses it."""
    R = sp.csr_matrix((np.ones(2, np.float32), np.array([0, 40000]), np.array([0, 1, 2])), shape=(2, 40000))
    with pytest.raises(nat.RPError, match="32767"):
        pack(R)
    R = sp.csr_matrix((np.full(2, 0.5, np.float32), np.array([0, 19999]), np.array([0, 1, 2])), shape=(2, 20000))
    info, _ = pack(R)
    assert info.layout == nat.RP_LAYOUT_GENERIC
    with pytest.raises(nat.RPError, match="packed"):
        pack(R, nat.RP_LAYOUT_PACKED)
    R = sp.csr_matrix((np.full(2, 0.5, np.float32), np.array([0, 16383]), np.array([0, 1, 2])), shape=(2, 16384))
    info, _ = pack(R)
    assert info.layout == nat.RP_LAYOUT_PACKED
