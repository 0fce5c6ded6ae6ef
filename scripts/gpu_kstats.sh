#!/bin/bash
# Per-kernel times (rocprofv3 kernel trace + stats) of bench.py runs; each variant in its own run.
# VARIANTS: "name|env assignments|bench args;..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  IFS='|' read -r name envs args <<< "$v"
  ( export $envs; timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/ks_$name -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline $args > gpurun_out/ks_$name.json 2> gpurun_out/ks_$name.err ) || { tail -20 gpurun_out/ks_$name.err; exit 5; }
  f=$(find gpurun_out/ks_$name -name '*kernel_stats.csv' | head -1)
  echo "== $name $(python3 -c "import json;d=json.load(open('gpurun_out/ks_$name.json'));print(round(d['ms_per_step'],2),'ms/step', d['verified']['sample_bitexact_vs_oracle'])")"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>4} avg_ms={float(r['AverageNs'])/1e6:8.3f} pct={float(r['Percentage']):5.1f}")
PY
done
