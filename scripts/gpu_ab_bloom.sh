#!/bin/bash
# A/B: Bloom check with four LDS loads in flight (librp_bloom.so) vs the current library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=randomprojection_amd
LIBS="$L/librp.so $L/librp_bloom.so $L/librp.so $L/librp_bloom.so" bash scripts/gpu_ab_ks.sh || exit $?
LIBS="$L/librp.so $L/librp_bloom.so" ARGS="--dist powerlaw" bash scripts/gpu_ab_ks.sh
