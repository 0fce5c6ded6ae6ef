#!/bin/bash
# round-3: libsvm tests + the boundary-3 line after vectorising line_count_kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_libsvm.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lsv2_tests.log 2>&1
rc=$?
tail -2 gpurun_out/lsv2_tests.log
[ $rc -ne 0 ] && { grep -n "Error\|FAILED" gpurun_out/lsv2_tests.log | head -8; exit $rc; }
timeout -k 10 300 python -u bench.py --boundary libsvm --steps 3 --warmup 1 > gpurun_out/r03_bench_libsvm2.json 2> gpurun_out/r03_bench_libsvm2.err || { tail -20 gpurun_out/r03_bench_libsvm2.err; exit 5; }
python3 -c "import json;d=json.load(open('gpurun_out/r03_bench_libsvm2.json'));print(round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],1), 'ms', d['verified'])"
