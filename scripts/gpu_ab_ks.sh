#!/bin/bash
# A/B of librp builds with per-kernel times: each library (bench.py --lib) in its own rocprofv3
# --kernel-trace --stats run; prints ms/step, the sample check and the top kernels.
#   LIBS="randomprojection_amd/librp_alt_a.so randomprojection_amd/librp_alt_b.so" ARGS="" bash scripts/gpu_ab_ks.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for lib in $LIBS; do
  i=$((i + 1))
  name=$(basename $lib .so)_$i
  timeout -k 10 ${BENCH_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/ks_$name -o run -- python3 bench.py --lib $lib --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${ARGS:-} > gpurun_out/ks_$name.json 2> gpurun_out/ks_$name.err || { tail -20 gpurun_out/ks_$name.err; exit 5; }
  f=$(find gpurun_out/ks_$name -name '*kernel_stats.csv' | head -1)
  echo "== $name $(python3 -c "import json;d=json.load(open('gpurun_out/ks_$name.json'));print(round(d['ms_per_step'],3),'ms/step', d['verified']['sample_bitexact_vs_oracle'], d['config']['nnz_out'])")"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:7]:
    print(f"  {r['Name'][:50]:50s} calls={r['Calls']:>4} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
PY
done
