"""bench.py's N-rank launch contract (BASELINE.json metric at 1/2/4/8 GPUs): --gpus must agree with
a launcher's WORLD_SIZE, never silently measuring another number of GPUs. Runs before any GPU or
torch import, so it is a CPU test."""
import os
import subprocess
import sys

from conftest import ROOT


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e, capture_output=True,
                          text=True, timeout=60)


def test_mismatched_world_size_fails_loudly():
    r = _bench(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
