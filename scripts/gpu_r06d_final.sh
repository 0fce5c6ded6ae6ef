#!/bin/bash
# Final round-6 check of the committed build (after the container rebuild): smoke(), the default
# bench line, and the whole -m gpu suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06d_smoke.log 2>&1 || { tail -5 gpurun_out/r06d_smoke.log; exit 3; }
tail -1 gpurun_out/r06d_smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06d_bench.json 2> gpurun_out/r06d_bench.err || { tail -5 gpurun_out/r06d_bench.err; exit 4; }
tail -c 400 gpurun_out/r06d_bench.json; echo
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r06d_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06d_gpu_tests.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/r06d_gpu_tests.log | grep -v PASSED | head -20
exit $rc
