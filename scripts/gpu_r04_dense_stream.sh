#!/bin/bash
# round 4 dense lines: resident GEMM + streamed 10M-row pass (ring of host chunks) for bf16 and f32,
# resident f64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in bf16 fp32; do
  timeout -k 10 400 python -u scripts/bench_dense.py --compute $c > gpurun_out/r04_dense_$c.json 2> gpurun_out/r04_dense_$c.err || { tail -20 gpurun_out/r04_dense_$c.err; exit 6; }
  cat gpurun_out/r04_dense_$c.json | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$c', d.get('metric','')[:60], round(d.get('value',0),1), d.get('unit'), d.get('roofline',{}).get('achieved'), d.get('full_pass_s', d.get('implied_full_pass_s')))"
done
timeout -k 10 300 python -u scripts/bench_dense.py --compute fp64 --no-stream > gpurun_out/r04_dense_fp64.json 2> gpurun_out/r04_dense_fp64.err || { tail -20 gpurun_out/r04_dense_fp64.err; exit 6; }
cat gpurun_out/r04_dense_fp64.json | head -c 600
