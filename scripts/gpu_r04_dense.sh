#!/bin/bash
# round 4: dense GEMM tests (every variant), then A/B of variant 11 (four-stage ring) vs 12 (ring with
# the next K-tile's fragments read ahead), bf16 and f32, twice each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dz_tests.log 2>&1
rc=$?
tail -2 gpurun_out/dz_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/dz_tests.log | head -8; exit $rc; }
for c in bf16 fp32; do for v in 11 12 11 12; do
  timeout -k 10 300 python -u scripts/bench_dense.py --compute $c --no-stream --variant $v > gpurun_out/dz_${c}_v$v.json 2> gpurun_out/dz_${c}_v$v.err || { tail -20 gpurun_out/dz_${c}_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/dz_${c}_v$v.json'));print('$c v$v', round(d['roofline']['achieved'],1), 'TF', d.get('rel_err_vs_fp64_same_operands',{}).get('librp'))"
done; done
