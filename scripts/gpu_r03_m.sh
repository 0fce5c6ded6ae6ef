#!/bin/bash
# round-3 session M: one-pass staging (segment reserves + claimed runs, no count pass) — staged,
# parity and full-size GPU tests, then per-kernel A/B against the previous build on configs[1].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
  -k "not configs3_full" --timeout 400 --timeout-method thread > gpurun_out/m_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/m_tests.log | tail -3; tail -2 gpurun_out/m_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED\|assert" gpurun_out/m_tests.log | head -12; exit $rc; }
LIBS="randomprojection_amd/librp_alt_base.so randomprojection_amd/librp.so" bash scripts/gpu_r03_j.sh
