#!/bin/bash
# configs[3] filtered tile pipeline: parity tests, then the cfg4 bench filtered and unfiltered with
# per-kernel times (rocprofv3 kernel stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_filter.py tests/test_gpu_longrow.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1
rc=$?
tail -2 gpurun_out/f_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED\|assert" gpurun_out/f_tests.log | head -20; exit $rc; }
for f in ${FILTERS:-1 0}; do
  LIBS="randomprojection_amd/librp.so" ARGS="--config cfg4 --filter $f" STEPS=${STEPS:-3} BENCH_TIMEOUT=600 bash scripts/gpu_ab_ks.sh || exit $?
done
