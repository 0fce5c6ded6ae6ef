#!/bin/bash
# A/B of librp builds on configs[3]-shaped rows (cfg4 bench, ROWS rows), filtered and unfiltered,
# per-kernel times; LIBS as for gpu_ab_ks.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${FILTERS:-1 0}; do
  LIBS="$LIBS" ARGS="--config cfg4 --rows ${ROWS:-20000000} --filter $f" STEPS=${STEPS:-3} BENCH_TIMEOUT=${BENCH_TIMEOUT:-150} bash scripts/gpu_ab_ks.sh || exit $?
done
