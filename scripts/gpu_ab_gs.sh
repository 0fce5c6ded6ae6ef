#!/bin/bash
# A/B: grid-stride wave kernel (gs), plain slot stores (plain), both (gsplain) vs the current library on
# configs[1] uniform / power-law; then the dense wide-ring bf16 variant (14, librp_dw.so) vs 11
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=randomprojection_amd
for v in 14 11 14 11; do
  timeout -k 10 300 python -u scripts/bench_dense.py --compute bf16 --no-stream --variant $v --lib $L/librp_dw.so > gpurun_out/dw_v$v.json 2> gpurun_out/dw_v$v.err || { tail -20 gpurun_out/dw_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/dw_v$v.json'));print('bf16 v$v', round(d['roofline']['achieved'],1), 'TF', d.get('rel_err_vs_fp64_same_operands',{}).get('librp'))"
done
LIBS="$L/librp.so $L/librp_gs.so $L/librp_plain.so $L/librp_gsplain.so $L/librp.so $L/librp_gs.so $L/librp_plain.so $L/librp_gsplain.so" bash scripts/gpu_ab_ks.sh || exit $?
LIBS="$L/librp.so $L/librp_gs.so $L/librp_plain.so $L/librp_gsplain.so" ARGS="--dist powerlaw" bash scripts/gpu_ab_ks.sh
