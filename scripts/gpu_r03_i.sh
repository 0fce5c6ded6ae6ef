#!/bin/bash
# round-3 session I: compacting staged gather (row-lane pipeline) — staged + parity + configs[1/2]
# full-size tests, then A/B against the previous build on configs[1], then in-kernel stage stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -k "not configs3_full" --timeout 400 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r03i_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/r03i_tests.log | head -8; exit $rc; }
LIBS="randomprojection_amd/librp_alt_base.so randomprojection_amd/librp.so randomprojection_amd/librp_alt_base.so randomprojection_amd/librp.so" \
  bash scripts/gpu_ab.sh || exit 4
timeout -k 10 300 python -u scripts/stage_stamps.py --rows 119705032 --p 4096 --lpr --staging on > gpurun_out/r03i_stamps.log 2>&1 || { tail -5 gpurun_out/r03i_stamps.log; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/stamps.json'));print({k:(v if not isinstance(v,dict) else {a:round(b,2) for a,b in v.items()}) for k,v in d.items()})"
