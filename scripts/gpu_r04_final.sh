#!/bin/bash
# round-4 final session: the whole -m gpu suite on the final sources, then smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04_final_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04_final_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/r04_final_tests.log | head -12; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1 || { tail -20 gpurun_out/r04_smoke.log; exit 7; }
tail -1 gpurun_out/r04_smoke.log
