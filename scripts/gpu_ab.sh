#!/bin/bash
# A/B wall-clock of librp builds on one bench configuration, each build in its own process.
#   LIBS="randomprojection_amd/librp.so randomprojection_amd/librp_alt_x.so" ARGS="--config cfg4" bash scripts/gpu_ab.sh
# Optional TESTS="tests/test_gpu_longrow.py ..." runs those GPU tests first (default build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?
  tail -6 gpurun_out/ab_tests.log
  if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
i=0
for lib in $LIBS; do
  i=$((i + 1))
  timeout -k 10 ${BENCH_TIMEOUT:-300} python3 bench.py --lib $lib --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${ARGS:-} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -20 gpurun_out/ab_$i.err; exit 4; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_$i.json'));print('$lib', round(d['ms_per_step'],3), 'ms', d['verified'].get('sample_bitexact_vs_oracle'), d['config'].get('nnz_out'))"
done
