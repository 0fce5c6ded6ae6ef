#!/bin/bash
# GPU test session: the whole -m gpu suite (or TESTSEL), then smoke. Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTSEL="${TESTSEL:-}"
timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} ${TESTFILES:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -5; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
