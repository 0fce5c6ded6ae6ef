#!/bin/bash
# round-3 final session A: the whole -m gpu suite on the final sources, then configs[2] on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?
tail -3 gpurun_out/final_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/final_tests.log | head -12; exit $rc; }
timeout -k 10 300 python -u bench.py --config kdd9x --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_kdd9x.json 2> gpurun_out/r03_bench_kdd9x.err || { tail -20 gpurun_out/r03_bench_kdd9x.err; exit 4; }
cut -c1-300 gpurun_out/r03_bench_kdd9x.json
