#!/bin/bash
# Round-6 final build (whole-line unit slots): PMC session keyed to the build (summarised on the box so
# the bench line reads its traffic), the default bench line, the whole -m gpu suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06e SKIP_BENCH=1 PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --host-steps 0" bash scripts/gpu_profile.sh > gpurun_out/r06e_prof.log 2>&1 || { tail -5 gpurun_out/r06e_prof.log; exit 4; }
echo prof-done
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06e_bench.json 2> gpurun_out/r06e_bench.err || { tail -5 gpurun_out/r06e_bench.err; exit 5; }
tail -c 300 gpurun_out/r06e_bench.json; echo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06e_gpu_tests.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/r06e_gpu_tests.log | grep -v PASSED | head -20
exit $rc
