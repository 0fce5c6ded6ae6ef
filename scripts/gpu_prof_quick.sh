#!/bin/bash
# Quick per-kernel timing (rocprofv3 kernel trace) of bench.py in a given staging mode, plus the
# diagnostic stage stamps. Usage: MODE=on|off TAG=name bash scripts/gpu_prof_quick.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MODE="${MODE:-on}"; TAG="${TAG:-quick}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$TAG -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --staging $MODE > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 5; }
cut -d, -f1-4 gpurun_out/prof_$TAG/trace_kernel_stats.csv | head -6
if [ -n "${STAMPS+x}" ]; then
  timeout -k 10 300 python3 scripts/stage_stamps.py --staging $MODE --out gpurun_out/stamps_$TAG.json > gpurun_out/stamps_$TAG.log 2>&1 || { tail -20 gpurun_out/stamps_$TAG.log; exit 6; }
  cat gpurun_out/stamps_$TAG.json
fi
