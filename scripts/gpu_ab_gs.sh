#!/bin/bash
# A/B: grid-stride wave kernel (gs), plain slot stores (plain), both (gsplain) vs the current library,
# uniform and power-law configs[1]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=randomprojection_amd
LIBS="$L/librp.so $L/librp_gs.so $L/librp_plain.so $L/librp_gsplain.so $L/librp.so $L/librp_gs.so $L/librp_plain.so $L/librp_gsplain.so" bash scripts/gpu_ab_ks.sh || exit $?
LIBS="$L/librp.so $L/librp_gs.so $L/librp_plain.so $L/librp_gsplain.so" ARGS="--dist powerlaw" bash scripts/gpu_ab_ks.sh
