#!/bin/bash
# A/B of librp variants under abso/ against the package build on one box: wall-clock ms/step
# (scripts/gpu_ab.sh) and per-kernel averages (scripts/gpu_kstats.sh).
#   LIBS="abso/a.so abso/b.so" bash scripts/gpu_r06_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh && bash scripts/gpu_kstats.sh
