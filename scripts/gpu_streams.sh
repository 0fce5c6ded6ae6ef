#!/bin/bash
# boundaries 2 and 3 (host CSR stream, libsvm stream) with per-kernel times, then the libsvm timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS=randomprojection_amd/librp.so ARGS="--boundary libsvm" STEPS=3 bash scripts/gpu_ab_ks.sh || exit $?
LIBS=randomprojection_amd/librp.so ARGS="--boundary host" STEPS=3 bash scripts/gpu_ab_ks.sh || exit $?
[ -n "${TRACE:-}" ] && bash scripts/gpu_trace_libsvm.sh
exit 0
