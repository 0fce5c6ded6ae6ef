#!/bin/bash
# round-3 session B: padded staged runs (row-lane) and nontemporal A streams (tile pipeline) A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r03b_tests.log
[ $rc -ne 0 ] && exit $rc
for pair in "kdd|" "kdd|--dist powerlaw" "cfg4|--config cfg4"; do
  IFS='|' read -r name args <<< "$pair"
  for lib in randomprojection_amd/librp_alt_base.so randomprojection_amd/librp.so randomprojection_amd/librp_alt_nt.so; do
    [ "$name" != "cfg4" ] && [ "$lib" = "randomprojection_amd/librp_alt_nt.so" ] && continue
    RP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline $args > gpurun_out/b_${name}.json 2> gpurun_out/b_${name}.err || { tail -20 gpurun_out/b_${name}.err; exit 4; }
    python3 -c "import json;d=json.load(open('gpurun_out/b_${name}.json'));print('$name', '$lib'.split('/')[-1], round(d['ms_per_step'],3), 'ms', d['verified']['sample_bitexact_vs_oracle'], d['staged_this_call'])"
  done
done
