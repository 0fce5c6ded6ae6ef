#!/bin/bash
# round-3 session N: staged GPU tests, then per-kernel A/B of the one-pass staging on configs[1].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1
rc=$?
tail -2 gpurun_out/n_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED\|assert" gpurun_out/n_tests.log | head -12; exit $rc; }
LIBS="randomprojection_amd/librp_alt_base.so randomprojection_amd/librp.so" bash scripts/gpu_r03_j.sh
