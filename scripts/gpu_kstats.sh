#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of bench.py for the package build
# and every --lib variant: one block per build (kernel, calls, avg ms).
#   LIBS="variants/a.so" BENCH="--dist powerlaw" bash scripts/gpu_kstats.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for L in "" ${LIBS:-}; do
  n=$((n + 1))
  arg=""; [ -n "$L" ] && arg="--lib $L"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/ks_$n -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 ${BENCH:-} $arg > gpurun_out/ks_$n.json 2> gpurun_out/ks_$n.log || exit 9
  echo "== ${L:-package}"
  python3 - "$n" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/ks_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("lpr_", "spgemm", "defer", "slot_copy", "tile_heavy")):
            n = r["Name"].split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
            print(f"{n:28s} {r['Calls']:>5} {float(r['AverageNs'])/1e6:8.3f}")
PY
done
