#!/bin/bash
# round-3 session A: new GPU tests (configs[3] full size, libsvm stream, 2-rank host boundary), then the
# boundary-2 and boundary-3 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_libsvm.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -v -x --timeout 400 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03a_tests.log | tail -30; tail -5 gpurun_out/r03a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --boundary host --steps 3 --warmup 1 > gpurun_out/r03_bench_host.json 2> gpurun_out/r03_bench_host.err || { tail -20 gpurun_out/r03_bench_host.err; exit 4; }
cut -c1-400 gpurun_out/r03_bench_host.json
timeout -k 10 300 python -u bench.py --boundary libsvm --steps 3 --warmup 1 > gpurun_out/r03_bench_libsvm.json 2> gpurun_out/r03_bench_libsvm.err || { tail -20 gpurun_out/r03_bench_libsvm.err; exit 5; }
cut -c1-600 gpurun_out/r03_bench_libsvm.json
