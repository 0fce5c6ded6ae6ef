#!/bin/bash
# round-3 session K: per-kernel A/B of SpGEMM variants on configs[1] (gpu_r03_j.sh), then the dense
# ring-buffer GEMM (variant 11): its tests and bf16 / fp32 rates against variant 10 and hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k_dense_tests.log 2>&1
rc=$?
tail -3 gpurun_out/k_dense_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/k_dense_tests.log | head -8; exit $rc; }
for c in bf16 fp32; do for v in 10 11; do
  timeout -k 10 300 python -u scripts/bench_dense.py --compute $c --no-stream --variant $v > gpurun_out/k_dense_${c}_v$v.json 2> gpurun_out/k_dense_${c}_v$v.err || { tail -20 gpurun_out/k_dense_${c}_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/k_dense_${c}_v$v.json'));print('$c v$v', round(d['roofline']['achieved'],1), 'TF', d.get('rel_err_vs_fp64_same_operands'), d.get('library_comparison',{}).get('torch_hipblaslt'))"
done; done
bash scripts/gpu_r03_j.sh
