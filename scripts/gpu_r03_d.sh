#!/bin/bash
# round-3 session D: configs[3] bitmap-filter variants, dense f32/bf16 kernels + tests, configs[3] full size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_dense_tests.log 2>&1 || { tail -30 gpurun_out/r03d_dense_tests.log; exit 3; }
tail -2 gpurun_out/r03d_dense_tests.log
for c in bf16 fp32 fp64; do for v in 5 10; do [ "$c" = fp64 ] && [ "$v" = 5 ] && continue;
  timeout -k 10 300 python -u scripts/bench_dense.py --compute $c --no-stream --variant $v > gpurun_out/r03_dense_${c}_v$v.json 2> gpurun_out/r03_dense_${c}_v$v.err || { tail -20 gpurun_out/r03_dense_${c}_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/r03_dense_${c}_v$v.json'));print('dense $c v$v', round(d['roofline']['achieved'],1), 'TF', d['rel_err_vs_fp64_same_operands'], round(d['library_comparison']['torch_hipblaslt']['tflops'],1))"
done; done
for lib in randomprojection_amd/librp.so randomprojection_amd/librp_alt_bm2.so randomprojection_amd/librp_alt_bm2nt.so; do
  RP_LIB=$lib timeout -k 10 300 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/d_cfg4.json 2> gpurun_out/d_cfg4.err || { tail -20 gpurun_out/d_cfg4.err; exit 4; }
  python3 -c "import json;d=json.load(open('gpurun_out/d_cfg4.json'));print('cfg4', '$lib'.split('/')[-1], round(d['ms_per_step'],3), 'ms', d['verified']['sample_bitexact_vs_oracle'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -s -x -k configs3_full --timeout 500 --timeout-method thread > gpurun_out/r03d_cfg3.log 2>&1
rc=$?
grep -E "PASSED|FAILED|before configs|A ready" gpurun_out/r03d_cfg3.log | tail -6
exit $rc
