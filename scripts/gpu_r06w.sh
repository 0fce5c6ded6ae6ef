set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="abvar/head.so abvar/nolds.so" bash scripts/gpu_kstats.sh > gpurun_out/r06w_kstats.txt 2>&1 || { cat gpurun_out/r06w_kstats.txt; exit 6; }
grep "==\|copy\|partition\|gather\|wave" gpurun_out/r06w_kstats.txt
for f in 1 2 3; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/ks_$f.json').read().strip().splitlines()[-1]); print($f, d['ms_per_step'], d['value'])"; done
