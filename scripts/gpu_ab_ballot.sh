#!/bin/bash
# A/B: wave-kernel step prefix from bit-plane ballots (librp_ballot.so) vs the DPP scan
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=randomprojection_amd
LIBS="$L/librp.so $L/librp_ballot.so $L/librp.so $L/librp_ballot.so" bash scripts/gpu_ab_ks.sh
