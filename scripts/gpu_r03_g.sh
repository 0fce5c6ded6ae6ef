#!/bin/bash
# round-3 session G: long-row wave pipeline v2 (flat tile loads): tests, configs[3] wave vs tile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_longrow.py -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/r03g_longrow.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03g_longrow.log | tail -8
[ $rc -ne 0 ] && exit $rc
for pipe in longrow tile; do
  timeout -k 10 300 python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --pipeline $pipe > gpurun_out/g_cfg4_$pipe.json 2> gpurun_out/g_cfg4_$pipe.err || { tail -20 gpurun_out/g_cfg4_$pipe.err; exit 4; }
  python3 -c "import json;d=json.load(open('gpurun_out/g_cfg4_$pipe.json'));print('cfg4 $pipe', round(d['ms_per_step'],3), 'ms', d['verified']['sample_bitexact_vs_oracle'], d['deferred_tiles'], d['tiles'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_g_cfg4 -o t -- python3 bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --pipeline longrow > gpurun_out/prof_g_cfg4.log 2>&1 || { tail -20 gpurun_out/prof_g_cfg4.log; exit 5; }
cut -d, -f1-4 gpurun_out/prof_g_cfg4/t_kernel_stats.csv | head -6
