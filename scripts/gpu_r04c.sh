#!/bin/bash
# filtered tile pipeline: its parity tests, then cfg4 benches (20M rows, then the full 200M) with
# per-kernel times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_filter.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/f_tests.log 2>&1
rc=$?
tail -2 gpurun_out/f_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED\|assert" gpurun_out/f_tests.log | head -20; exit $rc; }
LIBS="${LIBS:-randomprojection_amd/librp.so}" FILTERS="${FILTERS:-1}" bash scripts/gpu_ab_cfg4.sh || exit $?
[ -n "${FULL:-1}" ] && LIBS="${LIBS:-randomprojection_amd/librp.so}" FILTERS="${FILTERS:-1}" ROWS=200000000 BENCH_TIMEOUT=300 bash scripts/gpu_ab_cfg4.sh
