#!/bin/bash
# One GPU session: parity tests, smoke, bench. Stops at the first crash/timeout (exit >= 2 from
# pytest, or any non-zero from the other steps). Output under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTSEL="${TESTSEL:-not slow}"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$TESTSEL" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 4; }
  tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
fi
exit $rc
