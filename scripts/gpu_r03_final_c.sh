#!/bin/bash
# round-3 final session C: the whole -m gpu suite and smoke on the final sources.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final_c_tests.log 2>&1
rc=$?
tail -3 gpurun_out/final_c_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/final_c_tests.log | head -12; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
