"""librp and torch share one process and one device: either may touch the GPU first."""
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import sys; sys.path.insert(0, %r)
import numpy as np, scipy.sparse as sp
from randomprojection_amd import Projector, srp_matrix as sm
%s
P = Projector(sm.projection_operand(sm.sparse_random_matrix(64, 5000, random_state=123)))
import torch
x = torch.zeros(4, device="cuda")
print("ok", float(x.sum()))
"""


@pytest.mark.parametrize("lib", ["", "from randomprojection_amd import _native as nat; nat.load(%r)"])
def test_torch_after_librp(lib):
    """librp first (implicitly through Projector, or by an explicit load of the in-tree .so)."""
    if lib:
        lib = lib % (ROOT + "/randomprojection_amd/librp.so")
    r = subprocess.run([sys.executable, "-c", SCRIPT % (ROOT, lib)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok 0.0" in r.stdout, r.stderr[-2000:]
