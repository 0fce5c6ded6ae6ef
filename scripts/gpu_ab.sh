#!/bin/bash
# A/B timing of librp builds on one box: bench.py (configs[1] by default) for the package build and
# every --lib variant, interleaved ROUNDS times; one line per run: build id, ms/step, bit-exact check.
#   LIBS="variants/a.so variants/b.so" ROUNDS=2 BENCH="--dist powerlaw" bash scripts/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq "${ROUNDS:-2}"); do
  for L in "" ${LIBS:-}; do
    arg=""; [ -n "$L" ] && arg="--lib $L"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-steps 0 ${BENCH:-} $arg 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${L:-package}', d['librp']['build_id'], round(d['ms_per_step'], 3), d['verified']['sample_bitexact_vs_oracle'])" \
      || exit 9
  done
done
