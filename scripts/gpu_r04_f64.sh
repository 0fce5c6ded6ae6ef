#!/bin/bash
# f64 dense: tests (ring default + two-buffer variant 10), then both kernels' TFLOP/s twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dz_tests.log 2>&1
rc=$?
tail -2 gpurun_out/dz_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/dz_tests.log | head -8; exit $rc; }
for v in -1 10 -1 10; do
  timeout -k 10 300 python -u scripts/bench_dense.py --compute fp64 --no-stream --variant $v > gpurun_out/dz_fp64_v$v.json 2> gpurun_out/dz_fp64_v$v.err || { tail -20 gpurun_out/dz_fp64_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/dz_fp64_v$v.json'));print('fp64 v$v', round(d['roofline']['achieved'],2), 'TF', d.get('rel_err_vs_fp64_same_operands',{}))"
done
