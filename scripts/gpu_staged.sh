#!/bin/bash
# Staged-gather session: parity tests for both gather modes, then the full-size bench in each mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not slow" > gpurun_out/pytest_staged.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_staged.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for mode in on off; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --staging $mode > gpurun_out/bench_$mode.json 2> gpurun_out/bench_$mode.err || { tail -30 gpurun_out/bench_$mode.err; exit 4; }
  cat gpurun_out/bench_$mode.json
done
