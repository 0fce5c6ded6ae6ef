#!/bin/bash
# round-3 final session B: staged GPU tests + smoke on the final sources, then the configs[1] line and
# its profiles (PART 1: bench with the CPU baseline, kernel trace, PMC passes keyed to the sources).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_fullsize.py -m gpu -x -q -k "not configs3_full" --timeout 300 --timeout-method thread > gpurun_out/fb_tests.log 2>&1
rc=$?
tail -2 gpurun_out/fb_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/fb_tests.log | head -8; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 5
PART=1 bash scripts/gpu_r03_lines.sh
