#!/bin/bash
# round-3 session P: dense ring depth A/B + configs[1] wave states (gpu_r03_dense.sh), then the
# software-pipelined gather A/B on configs[1].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r03_dense.sh || exit $?
LIBS="randomprojection_amd/librp.so randomprojection_amd/librp_alt_v7.so randomprojection_amd/librp.so randomprojection_amd/librp_alt_v7.so" bash scripts/gpu_r03_o.sh
