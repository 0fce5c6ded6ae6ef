"""Test configuration. `-m "not gpu"` runs here (CPU only); `-m gpu` runs on an MI355X box."""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden_v1.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


@pytest.fixture(scope="session")
def golden():
    return np.load(GOLDEN, allow_pickle=False)


def golden_csr(g, prefix):
    return sp.csr_matrix((g[prefix + "_data"], g[prefix + "_indices"], g[prefix + "_indptr"]),
                         shape=tuple(g[prefix + "_shape"]))


def golden_R(g, which):
    """The projection operand the recipe uses: components_.T (CSC), f32 for R1, f64 for R2."""
    if which == 1:
        return golden_csr(g, "comp1").T.astype(np.float32)
    return golden_csr(g, "comp2").T


def same_bits(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))
