#!/bin/bash
# bench.py (configs[1] by default) under several argument sets, interleaved ROUNDS times; one line
# per run: the argument set, build id, ms/step, bit-exact check.
#   ARGSETS="--chunk-streams 1|--lpr-chunk-rows 30000000" ROUNDS=2 bash scripts/gpu_bench_args.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
IFS='|' read -ra SETS <<< "${ARGSETS:-}"
for r in $(seq "${ROUNDS:-2}"); do
  for A in "" "${SETS[@]}"; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-steps 0 ${BENCH:-} $A 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[${A:-default}]', d['librp']['build_id'], round(d['ms_per_step'], 3), d['verified']['sample_bitexact_vs_oracle'])" \
      || exit 9
  done
done
