#!/bin/bash
# round-3 session C: session B's A/B (padded runs, nontemporal tile loads), then the dist rehearsal,
# the full-size tests and the boundary-2/3 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_r03_b.sh || exit $?
for v in 5 10; do timeout -k 10 300 python -u scripts/bench_dense.py --compute bf16 --no-stream --variant $v > gpurun_out/r03_dense_v$v.json 2> gpurun_out/r03_dense_v$v.err || { tail -20 gpurun_out/r03_dense_v$v.err; exit 6; }; python3 -c "import json;d=json.load(open('gpurun_out/r03_dense_v$v.json'));print('dense v$v', round(d['roofline']['achieved'],1), 'TF', d['rel_err_vs_fp64_same_operands'])"; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -v -x --timeout 400 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03c_tests.log | tail -12; tail -3 gpurun_out/r03c_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --boundary host --steps 3 --warmup 1 > gpurun_out/r03_bench_host.json 2> gpurun_out/r03_bench_host.err || { tail -20 gpurun_out/r03_bench_host.err; exit 4; }
cut -c1-300 gpurun_out/r03_bench_host.json
timeout -k 10 300 python -u bench.py --boundary libsvm --steps 3 --warmup 1 > gpurun_out/r03_bench_libsvm.json 2> gpurun_out/r03_bench_libsvm.err || { tail -20 gpurun_out/r03_bench_libsvm.err; exit 5; }
cut -c1-300 gpurun_out/r03_bench_libsvm.json
for v in 5 10; do
  timeout -k 10 300 python -u scripts/bench_dense.py --compute bf16 --no-stream --variant $v > gpurun_out/r03_dense_v$v.json 2> gpurun_out/r03_dense_v$v.err || { tail -20 gpurun_out/r03_dense_v$v.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/r03_dense_v$v.json'));print('dense v$v', round(d['roofline']['achieved'],1), 'TF', d['rel_err_vs_fp64_same_operands'], d['library_comparison']['torch_hipblaslt'])"
done
