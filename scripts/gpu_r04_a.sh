#!/bin/bash
# round-4 session A: distributed + staged + parity GPU tests, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_staged.py tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/a_tests.log 2>&1
rc=$?
tail -3 gpurun_out/a_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/a_tests.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err || { tail -20 gpurun_out/a_bench.err; exit 4; }
cut -c1-600 gpurun_out/a_bench.json
