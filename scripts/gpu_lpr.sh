#!/bin/bash
# Row-lane pipeline session: parity tests forced onto it, then configs[1] timings (direct / staged)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RP_PIPE=lpr
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_staged.py ${EXTRA_TESTS:-} -x -q --timeout 300 --timeout-method thread > gpurun_out/lpr_tests.log 2>&1
rc=$?
tail -15 gpurun_out/lpr_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for st in off on; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --staging $st --no-cpu-baseline ${BENCH_EXTRA:-} > gpurun_out/lpr_bench_$st.json 2> gpurun_out/lpr_bench_$st.err || { tail -20 gpurun_out/lpr_bench_$st.err; exit 4; }
  python3 -c "import json;d=json.load(open('gpurun_out/lpr_bench_$st.json'));print('$st', round(d['ms_per_step'],2), 'ms', d['verified'], d['deferred_tiles'])"
done
