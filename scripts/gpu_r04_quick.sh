#!/bin/bash
# quick GPU check: the staged / parity tests (or TESTS), then the default bench line with kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_staged.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?
tail -2 gpurun_out/q_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED\|assert" gpurun_out/q_tests.log | head -20; exit $rc; }
LIBS="randomprojection_amd/librp.so" ARGS="${ARGS:-}" bash scripts/gpu_ab_ks.sh
